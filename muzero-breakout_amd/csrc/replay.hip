// Replay ingest on the device (replay_buffer.py:96-165).
//
// The acting loop's sink already holds, per step t and env b, the recorded action, reward,
// visit counts, root value and frame (u8 gray code) of every env still live at t (a prefix of
// the episode), plus the episode's first frame g(s0). ReplayBuffer.save_observation_trajectory
// turns each trajectory of length L > K + 1 (train_torch.py:223-225) into L - K + 1 windows:
// 32 past actions, 32 frames (31 padding frames g(s0) + the records, so frames run one behind
// the actions), K future actions / rewards / visit counts / values, the reward sum and K
// n-step value targets with the reference's f32 op order and its discount**K quirk.
//   replay_plan_kernel  (one workgroup): per-env length, reward sum, window counts, exclusive scan;
//   replay_write_kernel (one workgroup per surviving window): writes the window into a FIFO ring
//                        of fixed-size rows (frames stay u8 codes: 10 KB per window at 16x20);
//   replay_states_kernel: gathers a batch of windows' frames as f32 grayscale (the learner's input).
#include "common.h"

namespace {

struct ReplayRecords {
  const uint8_t* action;   // [T][B]
  const float* reward;     // [T][B]
  const uint8_t* mask;     // [T][B] recorded (not prev_done)
  const int64_t* counts;   // [T][B][3]
  const float* value;      // [T][B]
  const uint8_t* frame;    // [T][B][HW]
  const uint8_t* frame0;   // [B][HW]
  int T, B, HW;
};

struct ReplayRing {
  int64_t* past_actions;   // [cap][hist]
  int64_t* future_actions; // [cap][K]
  uint8_t* states;         // [cap][hist][HW]
  float* rewards;          // [cap][K]
  float* counts;           // [cap][K][3]
  float* values;           // [cap][K]
  float* targets;          // [cap][K]
  float* reward_sum;       // [cap]
  int cap;
};

constexpr int PT = 1024;

// lengths / reward sums / window offsets of the B trajectories (min_len: trajectories with
// length <= min_len are skipped, train_torch.py:224)
__global__ __launch_bounds__(PT) void replay_plan_kernel(ReplayRecords r, int K, int min_len, int32_t* lens,
                                                         float* rsum, int32_t* offsets) {
  __shared__ int32_t part[PT];
  const int tid = threadIdx.x;
  const int per = (r.B + PT - 1) / PT;
  int mine = 0;
  for (int u = 0; u < per; ++u) {
    const int b = tid * per + u;
    if (b >= r.B) break;
    int L = 0;
    float s = 0.f;
    for (int t = 0; t < r.T; ++t) {  // the recorded steps are a prefix of the episode
      if (r.mask[(size_t)t * r.B + b]) {
        s = s + r.reward[(size_t)t * r.B + b];  // ObservationTrajectory.reward_sum (replay_buffer.py:34)
        ++L;
      }
    }
    lens[b] = L;
    rsum[b] = s;
    mine += L > min_len && L >= K ? L - K + 1 : 0;
  }
  part[tid] = mine;
  __syncthreads();
  for (int o = 1; o < PT; o <<= 1) {  // inclusive scan over the per-thread sums
    const int v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int run = part[tid] - mine;
  for (int u = 0; u < per; ++u) {
    const int b = tid * per + u;
    if (b >= r.B) break;
    offsets[b] = run;
    const int L = lens[b];
    run += L > min_len && L >= K ? L - K + 1 : 0;
  }
  if (tid == PT - 1) offsets[r.B] = part[PT - 1];
}

// one workgroup per window j in [j0, n): env by binary search of offsets, ring slot (head + j) % cap
__global__ __launch_bounds__(256) void replay_write_kernel(ReplayRecords r, ReplayRing g, const int32_t* __restrict__ lens,
                                                           const float* __restrict__ rsum,
                                                           const int32_t* __restrict__ offsets, int K, int hist,
                                                           const float* __restrict__ dpow, int head, int j0) {
  const int j = j0 + blockIdx.x;
  int lo = 0, hi = r.B;  // last b with offsets[b] <= j
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (offsets[mid] <= j) lo = mid; else hi = mid;
  }
  const int b = lo, s = j - offsets[b], L = lens[b];
  const size_t slot = ((size_t)head + j) % g.cap;
  const int tid = threadIdx.x;
  const size_t B = r.B;
  if (tid < hist) {  // actions[s + tid] of the padded list: 32 zeros, then the records
    const int i = s + tid;
    g.past_actions[slot * hist + tid] = i < hist ? 0 : (int64_t)r.action[(size_t)(i - hist) * B + b];
  } else if (tid < hist + K) {
    const int i = tid - hist, t = s + i;  // records [s, s + K) (the padded lists' [s + 32, s + 32 + K))
    g.future_actions[slot * K + i] = (int64_t)r.action[(size_t)t * B + b];
    g.rewards[slot * K + i] = r.reward[(size_t)t * B + b];
    g.values[slot * K + i] = r.value[(size_t)t * B + b];
    for (int a = 0; a < 3; ++a) g.counts[(slot * K + i) * 3 + a] = (float)r.counts[((size_t)t * B + b) * 3 + a];
    // n-step target (replay_buffer.py:137-151): bootstrap td_steps = 10 ahead, scaled by
    // discount**K; dpow[k] = f32(discount**k) (python double pow, host table), dpow[T + 1] = f32(discount**K)
    const int cur = s + i, boot = s + 10 + i;
    float v;
    if (boot < L) {
      v = r.value[(size_t)boot * B + b] * dpow[r.T + 1];
      for (int k = 0; k < boot - cur; ++k) v = v + dpow[k] * r.reward[(size_t)(cur + k) * B + b];
    } else {
      v = dpow[0] * r.reward[(size_t)cur * B + b];  // python 0.0 + the first term is that term
      for (int k = 1; k < L - cur; ++k) v = v + dpow[k] * r.reward[(size_t)(cur + k) * B + b];
    }
    g.targets[slot * K + i] = v;
  } else if (tid == hist + K) {
    g.reward_sum[slot] = rsum[b];
  }
  // frames: the padded states list = 31 x g(s0), then the recorded frames
  const int chunks = r.HW / 16;
  uint8_t* dst = g.states + slot * hist * r.HW;
  for (int c = tid; c < hist * chunks; c += 256) {
    const int f = c / chunks, q = c - f * chunks, i = s + f;
    const uint8_t* src = i < hist - 1 ? r.frame0 + (size_t)b * r.HW : r.frame + ((size_t)(i - (hist - 1)) * B + b) * r.HW;
    *reinterpret_cast<uint4*>(dst + (size_t)f * r.HW + q * 16) = *reinterpret_cast<const uint4*>(src + q * 16);
  }
}

// batch gather of window frames as f32 grayscale: out[n][hist][HW] = lut[code & 7]
__global__ __launch_bounds__(256) void replay_states_kernel(const uint8_t* __restrict__ states, const int32_t* __restrict__ slots,
                                                            const float* __restrict__ lut, float* __restrict__ out,
                                                            int hist, int HW) {
  const int n = blockIdx.x;
  const uint8_t* src = states + (size_t)slots[n] * hist * HW;
  float* dst = out + (size_t)n * hist * HW;
  float l[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) l[i] = lut[i];
  const int c4 = hist * HW / 4;
  for (int c = threadIdx.x; c < c4; c += 256) {
    const uint32_t w = reinterpret_cast<const uint32_t*>(src)[c];
    float4 v = {l[w & 7], l[(w >> 8) & 7], l[(w >> 16) & 7], l[(w >> 24) & 7]};
    reinterpret_cast<float4*>(dst)[c] = v;
  }
}

}  // namespace

extern "C" {

int mzba_replay_plan(const uint8_t* action, const float* reward, const uint8_t* mask, const int64_t* counts,
                     const float* value, const uint8_t* frame, const uint8_t* frame0, int T, int B, int HW, int K,
                     int min_len, int32_t* lens, float* rsum, int32_t* offsets, hipStream_t stream) {
  MZ_CHECK_ARG(T > 0 && B > 0 && HW > 0 && K > 0 && mask && reward && lens && rsum && offsets, -1);
  ReplayRecords r{action, reward, mask, counts, value, frame, frame0, T, B, HW};
  hipLaunchKernelGGL(replay_plan_kernel, dim3(1), dim3(PT), 0, stream, r, K, min_len, lens, rsum, offsets);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_replay_write(const uint8_t* action, const float* reward, const uint8_t* mask, const int64_t* counts,
                      const float* value, const uint8_t* frame, const uint8_t* frame0, int T, int B, int HW,
                      const int32_t* lens, const float* rsum, const int32_t* offsets, int n_windows,
                      int64_t* past_actions, int64_t* future_actions, uint8_t* states, float* rewards,
                      float* counts_out, float* values_out, float* targets, float* reward_sum, int cap, int head,
                      int K, int hist, const float* dpow, hipStream_t stream) {
  MZ_CHECK_ARG(T > 0 && B > 0 && HW % 16 == 0 && K > 0 && hist >= 2 && hist + K < 256 && cap > 0 &&
               head >= 0 && head < cap && n_windows >= 0, -1);
  MZ_CHECK_ARG(dpow && action && reward && counts && value && frame && frame0 && lens && rsum && offsets && past_actions &&
               future_actions && states && rewards && counts_out && values_out && targets && reward_sum, -1);
  if (n_windows == 0) return 0;
  ReplayRecords r{action, reward, mask, counts, value, frame, frame0, T, B, HW};
  ReplayRing g{past_actions, future_actions, states, rewards, counts_out, values_out, targets, reward_sum, cap};
  const int j0 = n_windows > cap ? n_windows - cap : 0;  // older windows would be evicted at once
  hipLaunchKernelGGL(replay_write_kernel, dim3(n_windows - j0), dim3(256), 0, stream, r, g, lens, rsum, offsets, K,
                     hist, dpow, head, j0);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_replay_states(const uint8_t* states, const int32_t* slots, int n, const float* lut8, float* out, int hist,
                       int HW, hipStream_t stream) {
  MZ_CHECK_ARG(states && slots && lut8 && out && n >= 0 && hist > 0 && (hist * HW) % 4 == 0, -1);
  if (n == 0) return 0;
  hipLaunchKernelGGL(replay_states_kernel, dim3(n), dim3(256), 0, stream, states, slots, lut8, out, hist, HW);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
