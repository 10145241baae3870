// Breakout environment kernels for gfx950.
//
// Two state representations, same rules (environment/parallel_breakout.py:107-254):
//  * "planes": the reference's f32 (B,3,H,W) binary image + ball_dx i64 / ball_dy f32.
//    Drop-in for BreakoutEnvironment.reset/step; one 64-lane wave per env.
//  * "compact": SoA per-env scalars + a brick bitmask over the brick rows; used by the
//    fused acting loop. Phase 1 = one thread per env (branchy scalar rules), phase 2 =
//    the workgroup renders its envs' uint8 gray-code frames with 16-B coalesced stores
//    and pushes them into the frame-history ring (train_torch.py:201-209, 259-293).
#include "common.h"

namespace {

struct RewardCfg { float paddle_hit, brick_hit, lost, won; };

// gray code of a pixel: bit0 paddle, bit1 ball, bit2 brick. The float value of a code is
// clamp((0.3f*p + 1.0f*b) + 0.6f*br, 0, 1) (train_torch.py:334-358), see gray_lut().
MZ_DEV uint8_t gray_code(bool paddle, bool ball, bool brick) {
  return (uint8_t)((paddle ? 1 : 0) | (ball ? 2 : 0) | (brick ? 4 : 0));
}

// ---------------------------------------------------------------- reset (planes)
__device__ void reset_params(int b, int B, int W, int pw, uint64_t seed, int episode, int env_offset,
                             const int32_t* params, int& off, int& col, int& row, int& dx) {
  if (params) {
    off = params[0 * B + b]; col = params[1 * B + b]; row = params[2 * B + b]; dx = params[3 * B + b];
    return;
  }
  uint32_t e = (uint32_t)(b + env_offset);
  int low = -6;
  int high = W - pw - (W / 2 - pw / 2 - 1);  // parallel_breakout.py:115
  off = low + mz_randbelow(e, MZ_STREAM_RESET, episode, 0, seed, (uint32_t)(high - low));
  col = 1 + mz_randbelow(e, MZ_STREAM_RESET, episode, 1, seed, (uint32_t)(W - 2));
  row = -3 + mz_randbelow(e, MZ_STREAM_RESET, episode, 2, seed, 2u);
  dx = mz_randbelow(e, MZ_STREAM_RESET, episode, 3, seed, 2u) == 0 ? -1 : 1;
}

__global__ void env_reset_planes_kernel(float* __restrict__ state, int64_t* __restrict__ ball_dx,
                                        float* __restrict__ ball_dy, int B, int H, int W, int pw,
                                        int brick_rows, uint64_t seed, int episode, int env_offset,
                                        const int32_t* __restrict__ params) {
  int b = blockIdx.x;
  int off, col, row, dx;
  reset_params(b, B, W, pw, seed, episode, env_offset, params, off, col, row, dx);
  int ppos = W / 2 - pw / 2 + off;  // :120
  int by = ((H + row) % H + H) % H;  // :128 negative index from the bottom
  int HW = H * W;
  float* s = state + (size_t)b * 3 * HW;
  for (int i = threadIdx.x; i < 3 * HW; i += blockDim.x) {
    int ch = i / HW, p = i - ch * HW, y = p / W, x = p - y * W;
    float v = 0.f;
    if (ch == 0) v = (y == H - 1 && x >= ppos && x < ppos + pw) ? 1.f : 0.f;
    else if (ch == 1) v = (y == by && x == col) ? 1.f : 0.f;
    else v = (y < brick_rows) ? 1.f : 0.f;
    s[i] = v;
  }
  if (threadIdx.x == 0) { ball_dx[b] = dx; ball_dy[b] = -1.0f; }
}

// ---------------------------------------------------------------- step (planes)
// One wave per env. Follows parallel_breakout.py:158-254 op for op.
__global__ __launch_bounds__(64) void env_step_planes_kernel(
    const float* __restrict__ state, float* __restrict__ next_state, const int64_t* __restrict__ action,
    uint8_t* __restrict__ done, int64_t* __restrict__ ball_dx, float* __restrict__ ball_dy,
    float* __restrict__ reward, float* __restrict__ valid, int B, int H, int W, int pw, RewardCfg rc,
    int32_t* __restrict__ err) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int HW = H * W;
  const float* sp = state + (size_t)b * 3 * HW;
  const float* sball = sp + HW;
  const float* sbrick = sp + 2 * HW;
  // paddle position = first argmax of the paddle plane's last row (:177)
  float best = -INFINITY; int bi = 0x7fffffff;
  for (int x = lane; x < W; x += 64) {
    float v = sp[(H - 1) * W + x];
    if (v > best || (v == best && x < bi)) { best = v; bi = x; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(best, o); int oi = __shfl_xor(bi, o);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  // ball position (:189) — exactly one ball per env is required
  int cnt = 0, bpos = -1;
  for (int p = lane; p < HW; p += 64) {
    if (sball[p] == 1.0f) { cnt++; bpos = p; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    int ob = __shfl_xor(bpos, o);
    bpos = bpos > ob ? bpos : ob;
  }
  if (cnt != 1) {
    if (lane == 0) atomicOr(err, 1);
    return;
  }
  const int y = bpos / W, x = bpos - (bpos / W) * W;
  const int64_t a = action[b];
  int pnew = bi + (a == 0 ? -1 : (a == 2 ? 1 : 0));
  pnew = pnew < 0 ? 0 : (pnew > W - pw ? W - pw : pnew);  // :178-179
  const float ball_x = (float)x, ball_y = (float)y;
  int64_t dx = ball_dx[b];
  float dy = ball_dy[b];
  const bool wall = (ball_x + (float)dx < 0.f) || (ball_x + (float)dx >= (float)W);  // :195
  if (wall) dx = -dx;
  float ny = ball_y + dy;        // :198
  float nx = ball_x + (float)dx;  // :199
  const bool missed = ny >= (float)H;  // :202
  float r = 0.f;
  if (missed) r = rc.lost;
  bool dn = (done[b] != 0) || missed;  // :204
  if (dn) { dx = 0; dy = 0.f; }       // :207-208
  if (missed) ny = 0.f;                // :209
  if (ny < 0.f) { dy = dy * -1.0f; ny = ball_y; }  // :213-214
  const float old_dy = dy;                        // :217
  const int ix = (int)nx;
  const int bx = ix - (ix % 2);  // :218 (nx >= 0)
  const int iy = (int)ny;        // in [0, H) here
  const bool brick = !dn && sbrick[iy * W + bx] == 1.0f;  // :219 (bricks of done envs cleared)
  if (brick) dy = -old_dy;                                // :220
  if (brick) { ny = ball_y - old_dy; r = r + rc.brick_hit; }  // :224-226
  const bool hit = (ny == (float)(H - 1)) && ix >= pnew && ix < pnew + pw;  // :229-234
  if (hit) { dy = -dy; r = r + rc.paddle_hit; }                             // :235-239
  const int fy = (((int)ny) % H + H) % H;  // :243 row -1 wraps to H-1
  const int clr0 = iy * W + bx, clr1 = iy * W + ((bx + 1) % W);
  // finished = no bricks left after the unconditional clear (:221-222, :246)
  int any = 0;
  if (!dn) {
    for (int p = lane; p < HW; p += 64) any |= (sbrick[p] != 0.f && p != clr0 && p != clr1) ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) any |= __shfl_xor(any, o);
  const bool finished = any == 0;
  const bool dfin = dn || finished;  // :247
  if (finished != missed) r = r + rc.won;  // :250
  float* np_ = next_state + (size_t)b * 3 * HW;
  for (int p = lane; p < HW; p += 64) {
    const int py = p / W, px = p - py * W;
    float pv = dfin ? 0.f : (py == H - 1 ? ((px >= pnew && px < pnew + pw) ? 1.f : 0.f) : sp[p]);
    float bv = (py == fy && px == ix) ? 1.f : 0.f;
    float kv = dfin ? 0.f : ((p == clr0 || p == clr1) ? 0.f : sbrick[p]);
    np_[p] = pv; np_[HW + p] = bv; np_[2 * HW + p] = kv;
  }
  if (lane == 0) {
    done[b] = dfin ? 1 : 0;
    ball_dx[b] = dx;
    ball_dy[b] = dy;
    reward[b] = r;
    valid[b * 3 + 0] = pnew == 0 ? 0.f : 1.f;  // :153
    valid[b * 3 + 1] = 1.f;
    valid[b * 3 + 2] = (pnew + pw >= W) ? 0.f : 1.f;  // :154
  }
}

// ---------------------------------------------------------------- compact state
// SoA compact state (global env b):
//   paddle[b] (i32, left column; plane empty <=> done), bx/by (i32), dx (i32), dy (f32),
//   done (u8), bricks[b*nw .. b*nw+nw) (u64 bitmask, bit = row*W + col, rows < brick_rows)
struct Compact {
  int32_t* paddle; int32_t* bx; int32_t* by; int32_t* dx; float* dy; uint8_t* done; uint64_t* bricks; int nw;
};

// History ring (train_torch.py:313-332 pad, :204-209 record, :259-293 read):
//   frames[b][L-1][HW] u8 gray codes, actions[b][L] u8, hlen[b] = records pushed so far.
// cur_src (optional, single-write mode): cur_src[b] = 1 when env b's current frame is the
// ring's newest entry (it was recorded by the last step / reset), 0 when it is cur_frame[b]
// (a done env: history frozen, frame live). Every frame is then written to HBM exactly once.
// cur_src == NULL: cur_frame always holds the current frame (a recorded frame is written twice).
struct History { uint8_t* frames; uint8_t* actions; int32_t* hlen; int L; uint8_t* cur_src; };

// where env b's current frame lives (see History)
MZ_DEV const uint8_t* current_frame_ptr(const uint8_t* cur_frame, const History& h, size_t b, int HW) {
  if (h.cur_src && h.cur_src[b]) {
    const int slot = (h.hlen[b] + h.L - 2) % (h.L - 1);  // newest ring entry
    return h.frames + (b * (h.L - 1) + slot) * (size_t)HW;
  }
  return cur_frame + b * (size_t)HW;
}

// Trajectory sink (replay_buffer.py:17-35 ObservationTrajectory.add_observation),
// per acting step t: rec_action[t][b] u8, rec_reward[t][b] f32, rec_mask[t][b] u8; the
// recorded frame is cur_frame (written to rec_frame[t][b][HW] when non-null).
struct Sink { uint8_t* action; float* reward; uint8_t* mask; uint8_t* frame; };

__global__ void env_reset_compact_kernel(Compact cs, uint8_t* __restrict__ cur_frame, History hist, int pad_action, int B,
                                         int H, int W, int pw, int brick_rows, uint64_t seed, int episode,
                                         int env_offset, const int32_t* __restrict__ params) {
  // one block per env: scalars by thread 0, frame + history pad by the block
  const int b = blockIdx.x;
  int off, col, row, dx;
  reset_params(b, B, W, pw, seed, episode, env_offset, params, off, col, row, dx);
  const int ppos = W / 2 - pw / 2 + off;
  const int by = ((H + row) % H + H) % H;
  const int HW = H * W;
  if (threadIdx.x == 0) {
    cs.paddle[b] = ppos; cs.bx[b] = col; cs.by[b] = by; cs.dx[b] = dx; cs.dy[b] = -1.0f; cs.done[b] = 0;
    hist.hlen[b] = 0;
    if (hist.cur_src) hist.cur_src[b] = 1;  // current = g(s0) = the ring's newest pad frame
  }
  for (int w = threadIdx.x; w < cs.nw; w += blockDim.x) {
    uint64_t m = 0;
    for (int k = 0; k < 64; ++k) {
      int bit = w * 64 + k;
      if (bit < brick_rows * W) m |= (1ull << k);
    }
    cs.bricks[(size_t)b * cs.nw + w] = m;
  }
  uint8_t* cf = cur_frame + (size_t)b * HW;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    int y = p / W, x = p - y * W;
    uint8_t c = gray_code(y == H - 1 && x >= ppos && x < ppos + pw, y == by && x == col, y < brick_rows);
    if (!hist.cur_src) cf[p] = c;
    for (int k = 0; k < hist.L - 1; ++k) hist.frames[((size_t)b * (hist.L - 1) + k) * HW + p] = c;
  }
  for (int k = threadIdx.x; k < hist.L; k += blockDim.x) hist.actions[(size_t)b * hist.L + k] = (uint8_t)pad_action;
}

// one 16-B chunk of a rendered frame: a non-temporal store (written once, read by a later launch
// at most once: 84x84 B=4096 10.3 -> 8.6 us per graph-replayed step)
MZ_DEV void frame_store(uint8_t* p, uint4 v) {
#ifndef MZ_ENV_TEMPORAL
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
#else
  *reinterpret_cast<uint4*>(p) = v;
#endif
}

// Phase 1: one thread per env, all rules on the compact state (same op order as above).
// Phase 2: the block renders its E envs' frames (16 B per lane per store) and pushes
// them into the history ring when the env is recorded this step. E (<= 256) is chosen by the
// launcher so that the grid fills the chip and a block has ~1-4 stores per lane.
template <int MAXW>
__global__ __launch_bounds__(256, 8) void env_step_compact_kernel(
    Compact cs, const int64_t* __restrict__ action, float* __restrict__ reward, float* __restrict__ valid,
    uint8_t* __restrict__ cur_frame, History hist, Sink sink, int first_step_arg, int B, int H, int W, int pw,
    int brick_rows, RewardCfg rc, const int32_t* __restrict__ ctx, int E, int rec_flags) {
  // graph replay: the episode row t comes from the device context; the sink pointers are the
  // (T, B, ...) bases and row t is selected here; t == 0 is the first step.
  // Every load of phase 1 (ctx, the env's state, its history length, its action) is issued
  // unconditionally and before the first use of any of them: one memory round trip ahead of the
  // render stores, not three (a conditional paddle load behind `done`, the ctx load ahead of both
  // serialised them: 10.5 -> see DESIGN.md §3.3).
  // ctx[2] through a vector load (a VGPR zero index): a scalar load would put its round trip
  // ahead of the state loads (s_waitcnt lgkmcnt(0) also waits for the kernel arguments)
  int vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  // every kernel argument into SGPRs here: left to itself the compiler loads them in four
  // groups, each behind its own s_waitcnt (four scalar-cache round trips ahead of the first
  // state load)
  asm volatile("" ::"s"(cs.paddle), "s"(cs.bx), "s"(cs.by), "s"(cs.dx), "s"(cs.dy), "s"(cs.done), "s"(cs.bricks),
               "s"(cs.nw), "s"(action), "s"(reward), "s"(valid), "s"(cur_frame));
  asm volatile("" ::"s"(hist.frames), "s"(hist.actions), "s"(hist.hlen), "s"(hist.L), "s"(hist.cur_src),
               "s"(sink.action), "s"(sink.reward), "s"(sink.mask), "s"(sink.frame), "s"(ctx), "s"(E), "s"(B));
  const int ctx_t = ctx ? ctx[2 + vzero] : 0;
  __shared__ int s_paddle[256], s_bx[256], s_by[256];
  __shared__ uint64_t s_br[256][MAXW];
  __shared__ uint8_t s_done[256], s_rec[256];
  __shared__ int s_slot[256], s_slot_hl[256];
  const int t = threadIdx.x;
  const int b = blockIdx.x * E + t;
  const int nw = cs.nw;
  if (t < E && b < B) {
    const int hl = hist.hlen[b];
    const uint8_t done8 = cs.done[b];
    const int paddle_ld = cs.paddle[b];
    const int64_t a = action[b];
    const int x = cs.bx[b], y = cs.by[b];
    int dx = cs.dx[b];
    float dy = cs.dy[b];
    uint64_t br[MAXW];
#pragma unroll
    for (int w = 0; w < MAXW; ++w) br[w] = cs.bricks[(size_t)b * nw + (w < nw ? w : nw - 1)];
#pragma unroll
    for (int w = 0; w < MAXW; ++w) br[w] = w < nw ? br[w] : 0ull;
    const int first_step = ctx ? (ctx_t == 0) : first_step_arg;
    const bool was_done = done8 != 0;
    const int p0 = was_done ? 0 : paddle_ld;  // argmax of an empty row is 0 (:177)
    int pnew = p0 + (a == 0 ? -1 : (a == 2 ? 1 : 0));
    pnew = pnew < 0 ? 0 : (pnew > W - pw ? W - pw : pnew);
    const float ball_x = (float)x, ball_y = (float)y;
    const bool wall = (ball_x + (float)dx < 0.f) || (ball_x + (float)dx >= (float)W);
    if (wall) dx = -dx;
    float ny = ball_y + dy;
    float nx = ball_x + (float)dx;
    const bool missed = ny >= (float)H;
    float r = 0.f;
    if (missed) r = rc.lost;
    const bool dn = was_done || missed;
    if (dn) { dx = 0; dy = 0.f; }
    if (missed) ny = 0.f;
    if (ny < 0.f) { dy = dy * -1.0f; ny = ball_y; }
    const float old_dy = dy;
    const int ix = (int)nx;
    const int bxx = ix - (ix % 2);
    const int iy = (int)ny;
    bool brick = false;
    if (!dn && iy < brick_rows) {
      int bit = iy * W + bxx;
      brick = (br[bit >> 6] >> (bit & 63)) & 1ull;
    }
    if (brick) dy = -old_dy;
    if (iy < brick_rows) {  // unconditional clear of (iy,bxx),(iy,bxx+1)
      int b0 = iy * W + bxx, b1 = iy * W + ((bxx + 1) % W);
#pragma unroll
      for (int w = 0; w < MAXW; ++w) {
        if ((b0 >> 6) == w) br[w] &= ~(1ull << (b0 & 63));
        if ((b1 >> 6) == w) br[w] &= ~(1ull << (b1 & 63));
      }
    }
    if (brick) { ny = ball_y - old_dy; r = r + rc.brick_hit; }
    const bool hit = (ny == (float)(H - 1)) && ix >= pnew && ix < pnew + pw;
    if (hit) { dy = -dy; r = r + rc.paddle_hit; }
    const int fy = (((int)ny) % H + H) % H;
    uint64_t any = 0;
#pragma unroll
    for (int w = 0; w < MAXW; ++w) any |= br[w];
    const bool finished = dn || any == 0ull;
    const bool dfin = dn || finished;
    if (finished != missed) r = r + rc.won;
    if (dfin) {
#pragma unroll
      for (int w = 0; w < MAXW; ++w) br[w] = 0ull;
    }
    cs.paddle[b] = pnew; cs.bx[b] = ix; cs.by[b] = fy; cs.dx[b] = dx; cs.dy[b] = dy;
    cs.done[b] = dfin ? 1 : 0;
#pragma unroll
    for (int w = 0; w < MAXW; ++w) if (w < nw) cs.bricks[(size_t)b * nw + w] = br[w];
    reward[b] = r;
    valid[b * 3 + 0] = pnew == 0 ? 0.f : 1.f;
    valid[b * 3 + 1] = 1.f;
    valid[b * 3 + 2] = (pnew + pw >= W) ? 0.f : 1.f;
    // record iff not prev_done; at the first step prev_done aliases done (train_torch.py:179).
    // rec_flags (run_test_simulation, train_torch.py:594-598): bit 0 records every env, bit 1
    // records env 0's action for every env (the reference's action[0] there)
    const bool rec = (rec_flags & 1) ? true : (first_step ? !dfin : !was_done);
    const int64_t ra = (rec_flags & 2) ? action[0] : a;
    if (sink.action) {
      const size_t row = (size_t)ctx_t * B;  // ctx_t = 0 without a device context
      sink.action[row + b] = (uint8_t)ra; sink.reward[row + b] = r; sink.mask[row + b] = rec ? 1 : 0;
    }
    s_paddle[t] = dfin ? -1 : pnew; s_bx[t] = ix; s_by[t] = fy; s_done[t] = dfin; s_rec[t] = rec;
#pragma unroll
    for (int w = 0; w < MAXW; ++w) s_br[t][w] = br[w];
    if (rec) {
      hist.actions[(size_t)b * hist.L + (hl % hist.L)] = (uint8_t)ra;
      s_slot[t] = hl % (hist.L - 1);
      s_slot_hl[t] = hl;
    }
  }
  __syncthreads();
  // phase 2: render. Frame rows are HW bytes; lanes write 16 B (HW % 16 == 0 required).
  // A pixel's code depends on its index p alone: brick bit p of the mask (bit = row*W + col),
  // paddle iff p in [(H-1)*W + paddle, +pw), ball iff p == by*W + bx. So a 16-pixel chunk is
  // three 16-bit masks spread to bytes — no per-pixel division, no branch on the region.
  const int HW = H * W;
  const int chunks = HW / 16;
  const int nenv = min(E, B - (int)blockIdx.x * E);
  uint8_t* const sink_frame = sink.frame ? sink.frame + (size_t)ctx_t * B * HW : nullptr;
  const uint32_t inv_chunks = 0xffffffffu / (uint32_t)chunks + 1u;  // exact i / chunks for i < 2^32 / chunks
  for (int i = t; i < nenv * chunks; i += 256) {
    const int e = (int)__umulhi((uint32_t)i, inv_chunks), c = i - e * chunks;
    const int gb = blockIdx.x * E + e;
    const int p0 = c * 16;
    uint32_t brk16 = 0;
    if ((p0 >> 6) < nw) brk16 = (uint32_t)(s_br[e][p0 >> 6] >> (p0 & 48)) & 0xffffu;  // p0 % 16 == 0: one word
    const int plo = s_paddle[e] < 0 ? 0x7fff0000 : (H - 1) * W + s_paddle[e] - p0;
    const int lo = max(plo, 0), hi = min(plo + pw, 16);
    const uint32_t pad16 = lo < hi ? ((1u << hi) - 1u) & ~((1u << lo) - 1u) : 0u;
    const int bo = s_by[e] * W + s_bx[e] - p0;
    const uint32_t ball16 = (bo >= 0 && bo < 16) ? (1u << bo) : 0u;
    uint32_t wv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // nibble n -> 4 bytes holding n's bits: (n * 0x204081) & 0x01010101
      const uint32_t nb = ((brk16 >> (4 * q)) & 15u) * 0x204081u & 0x01010101u;
      const uint32_t nl = ((ball16 >> (4 * q)) & 15u) * 0x204081u & 0x01010101u;
      const uint32_t np = ((pad16 >> (4 * q)) & 15u) * 0x204081u & 0x01010101u;
      wv[q] = (nb << 2) | (nl << 1) | np;  // gray_code(paddle, ball, brick)
    }
    uint4 v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    if (sink_frame) frame_store(sink_frame + (size_t)gb * HW + c * 16, v);
    if (s_rec[e]) {
      frame_store(hist.frames + ((size_t)gb * (hist.L - 1) + s_slot[e]) * HW + c * 16, v);
      if (!hist.cur_src) frame_store(cur_frame + (size_t)gb * HW + c * 16, v);
    } else {
      frame_store(cur_frame + (size_t)gb * HW + c * 16, v);
    }
  }
  if (t < E && b < B) {
    if (s_rec[t]) hist.hlen[b] = s_slot_hl[t] + 1;  // phase 2 reads hlen only through s_slot
    if (hist.cur_src) hist.cur_src[b] = s_rec[t];
  }
}

// compact -> planes (for parity checks and the drop-in API)
__global__ void compact_to_planes_kernel(Compact cs, float* __restrict__ planes, int H, int W, int pw,
                                         int brick_rows) {
  const int b = blockIdx.x, HW = H * W;
  const bool dn = cs.done[b] != 0;
  const int pp = cs.paddle[b], bx = cs.bx[b], by = cs.by[b];
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    int y = p / W, x = p - y * W;
    float* o = planes + (size_t)b * 3 * HW;
    o[p] = (!dn && y == H - 1 && x >= pp && x < pp + pw) ? 1.f : 0.f;
    o[HW + p] = (y == by && x == bx) ? 1.f : 0.f;
    float k = 0.f;
    if (y < brick_rows) { int bit = y * W + x; k = ((cs.bricks[(size_t)b * cs.nw + (bit >> 6)] >> (bit & 63)) & 1ull) ? 1.f : 0.f; }
    o[2 * HW + p] = k;
  }
}

// grayscale from planes (train_torch.py:334-358), f32 out (B,1,H,W)
__global__ void grayscale_planes_kernel(const float* __restrict__ s, float* __restrict__ g, int B, int HW) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)B * HW) return;
  size_t b = i / HW, p = i - b * HW;
  const float* sp = s + b * 3 * HW;
  float v = (sp[p] * 0.3f + sp[HW + p] * 1.0f) + sp[2 * HW + p] * 0.6f;
  g[i] = fminf(fmaxf(v, 0.f), 1.f);
}

// Representation-net input (train_torch.py:259-293) from the history ring, NHWC with
// channel stride Cs (>= 2L, zero padded): c < L-1: ring frames oldest first; c == L-1:
// current frame; L <= c < 2L: action a/3 planes (oldest first).
template <typename T>
__global__ void build_rep_input_kernel(const uint8_t* __restrict__ cur_frame, History hist, T* __restrict__ out,
                                       int B, int HW, int Cs) {
  __shared__ float lut[8];
  if (threadIdx.x < 8) {
    int c = threadIdx.x;
    float pv = (c & 1) ? 1.f : 0.f, bv = (c & 2) ? 1.f : 0.f, kv = (c & 4) ? 1.f : 0.f;
    float v = (pv * 0.3f + bv * 1.0f) + kv * 0.6f;
    lut[c] = fminf(fmaxf(v, 0.f), 1.f);
  }
  __syncthreads();
  const int L = hist.L;
  const int CH = Cs / 8;  // 8-channel chunks per pixel: one 16-B (bf16) / 32-B (f32) store per thread
  const size_t n = (size_t)B * HW * CH;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t pix = i / CH;
    const int ch = (int)(i - pix * CH);
    const size_t b = pix / HW, p = pix - b * HW;
    const int hl = hist.hlen[b];
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = ch * 8 + j;
      float x = 0.f;
      if (c < L - 1) x = lut[hist.frames[(b * (L - 1) + ((hl + c) % (L - 1))) * HW + p] & 7];
      else if (c == L - 1) x = lut[current_frame_ptr(cur_frame, hist, b, HW)[p] & 7];
      else if (c < 2 * L) x = (float)hist.actions[b * L + ((hl + c - L) % L)] / 3.0f;
      v[j] = x;
    }
    T* o = out + pix * Cs + ch * 8;
    if constexpr (sizeof(T) == 2) {
      uint4 w;
      w.x = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
      w.y = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
      w.z = (uint32_t)f32_to_bf16(v[4]) | ((uint32_t)f32_to_bf16(v[5]) << 16);
      w.w = (uint32_t)f32_to_bf16(v[6]) | ((uint32_t)f32_to_bf16(v[7]) << 16);
      *reinterpret_cast<uint4*>(o) = w;
    } else {
      reinterpret_cast<float4*>(o)[0] = make_float4(v[0], v[1], v[2], v[3]);
      reinterpret_cast<float4*>(o)[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// materialise every env's current frame (single-write mode keeps it in the ring or cur_frame)
__global__ void current_frame_kernel(const uint8_t* __restrict__ cur_frame, History hist, uint8_t* __restrict__ out,
                                     int B, int HW) {
  const int b = blockIdx.x;
  const uint8_t* src = current_frame_ptr(cur_frame, hist, b, HW);
  for (int p = threadIdx.x; p < HW; p += blockDim.x) out[(size_t)b * HW + p] = src[p];
}

}  // namespace

static thread_local int g_block_envs = 0;  // 0 = automatic (mzba_env_set_block_envs, diagnostics)

// =============================================================================== C ABI
extern "C" {

int mzba_env_set_block_envs(int E) {
  MZ_CHECK_ARG(E >= 0 && E <= 256, -1);
  g_block_envs = E;
  return 0;
}

int mzba_env_reset_planes(float* state, int64_t* ball_dx, float* ball_dy, int B, int H, int W, int paddle_width,
                          int brick_rows, uint64_t seed, int episode, int env_offset, const int32_t* params,
                          hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && H > 3 && W > paddle_width && (W % 2) == 0, -1);
  hipLaunchKernelGGL(env_reset_planes_kernel, dim3(B), dim3(256), 0, stream, state, ball_dx, ball_dy, B, H, W,
                     paddle_width, brick_rows, seed, episode, env_offset, params);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_env_step_planes(const float* state, float* next_state, const int64_t* action, uint8_t* done,
                         int64_t* ball_dx, float* ball_dy, float* reward, float* valid, int B, int H, int W,
                         int paddle_width, const float* rewards4, int32_t* err, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && H > 3 && W > paddle_width && (W % 2) == 0 && rewards4 && err, -1);
  RewardCfg rc{rewards4[0], rewards4[1], rewards4[2], rewards4[3]};
  hipLaunchKernelGGL(env_step_planes_kernel, dim3(B), dim3(64), 0, stream, state, next_state, action, done, ball_dx,
                     ball_dy, reward, valid, B, H, W, paddle_width, rc, err);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_grayscale_planes(const float* state, float* gray, int B, int H, int W, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0, -1);
  size_t n = (size_t)B * H * W;
  hipLaunchKernelGGL(grayscale_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, state, gray,
                     B, H * W);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_env_reset_compact(int32_t* paddle, int32_t* bx, int32_t* by, int32_t* dx, float* dy, uint8_t* done,
                           uint64_t* bricks, int nw, uint8_t* cur_frame, uint8_t* cur_src, uint8_t* hist_frames,
                           uint8_t* hist_actions, int32_t* hist_len, int L, int B, int H, int W, int paddle_width,
                           int brick_rows, uint64_t seed, int episode, int env_offset, const int32_t* params,
                           int pad_action, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && L >= 2 && nw * 64 >= brick_rows * W && nw <= 4 && (H * W) % 16 == 0 && pad_action >= 0 &&
               pad_action < 3, -1);
  Compact cs{paddle, bx, by, dx, dy, done, bricks, nw};
  History h{hist_frames, hist_actions, hist_len, L, cur_src};
  hipLaunchKernelGGL(env_reset_compact_kernel, dim3(B), dim3(256), 0, stream, cs, cur_frame, h, pad_action, B, H, W,
                     paddle_width, brick_rows, seed, episode, env_offset, params);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_env_step_compact(int32_t* paddle, int32_t* bx, int32_t* by, int32_t* dx, float* dy, uint8_t* done,
                          uint64_t* bricks, int nw, const int64_t* action, float* reward, float* valid,
                          uint8_t* cur_frame, uint8_t* cur_src, uint8_t* hist_frames, uint8_t* hist_actions,
                          int32_t* hist_len, int L, uint8_t* rec_action, float* rec_reward, uint8_t* rec_mask, uint8_t* rec_frame,
                          int first_step, int B, int H, int W, int paddle_width, int brick_rows,
                          const float* rewards4, const int32_t* ctx, int rec_flags, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && L >= 2 && nw >= 1 && nw <= 4 && nw * 64 >= brick_rows * W && (H * W) % 16 == 0 &&
               H * W <= 65536 && rewards4, -1);  // H*W bound: the render loop's reciprocal division
  Compact cs{paddle, bx, by, dx, dy, done, bricks, nw};
  History h{hist_frames, hist_actions, hist_len, L, cur_src};
  Sink sk{rec_action, rec_reward, rec_mask, rec_frame};
  RewardCfg rc{rewards4[0], rewards4[1], rewards4[2], rewards4[3]};
  // envs per block: ~<= 4 16-B render stores per lane, and >= ~512 blocks when B allows
  const int chunks = H * W / 16;
  int E = 1;
  while (E < 256 && 2 * E * chunks <= 1024 && 2 * E * 512 <= B) E *= 2;
  if (g_block_envs > 0) E = g_block_envs;
  dim3 grid((B + E - 1) / E);
  if (nw == 1)
    hipLaunchKernelGGL(env_step_compact_kernel<1>, grid, dim3(256), 0, stream, cs, action, reward, valid, cur_frame,
                       h, sk, first_step, B, H, W, paddle_width, brick_rows, rc, ctx, E, rec_flags);
  else
    hipLaunchKernelGGL(env_step_compact_kernel<4>, grid, dim3(256), 0, stream, cs, action, reward, valid, cur_frame,
                       h, sk, first_step, B, H, W, paddle_width, brick_rows, rc, ctx, E, rec_flags);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_compact_to_planes(const int32_t* paddle, const int32_t* bx, const int32_t* by, const uint8_t* done,
                           const uint64_t* bricks, int nw, float* planes, int B, int H, int W, int paddle_width,
                           int brick_rows, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0, -1);
  Compact cs{(int32_t*)paddle, (int32_t*)bx, (int32_t*)by, nullptr, nullptr, (uint8_t*)done, (uint64_t*)bricks, nw};
  hipLaunchKernelGGL(compact_to_planes_kernel, dim3(B), dim3(256), 0, stream, cs, planes, H, W, paddle_width,
                     brick_rows);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_build_rep_input(const uint8_t* cur_frame, const uint8_t* cur_src, const uint8_t* hist_frames,
                         const uint8_t* hist_actions, const int32_t* hist_len, int L, void* out, int out_bf16, int B,
                         int HW, int Cs, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && Cs >= 2 * L && Cs % 8 == 0, -1);
  History h{(uint8_t*)hist_frames, (uint8_t*)hist_actions, (int32_t*)hist_len, L, (uint8_t*)cur_src};
  size_t n = (size_t)B * HW * (Cs / 8);
  unsigned grid = (unsigned)((n + 255) / 256);
  if (grid > 16384) grid = 16384;
  if (out_bf16)
    hipLaunchKernelGGL(build_rep_input_kernel<bf16_t>, dim3(grid), dim3(256), 0, stream, cur_frame, h,
                       (bf16_t*)out, B, HW, Cs);
  else
    hipLaunchKernelGGL(build_rep_input_kernel<float>, dim3(grid), dim3(256), 0, stream, cur_frame, h, (float*)out,
                       B, HW, Cs);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_env_current_frame(const uint8_t* cur_frame, const uint8_t* cur_src, const uint8_t* hist_frames,
                           const int32_t* hist_len, int L, uint8_t* out, int B, int HW, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && L >= 2 && HW > 0 && out, -1);
  History h{(uint8_t*)hist_frames, nullptr, (int32_t*)hist_len, L, (uint8_t*)cur_src};
  hipLaunchKernelGGL(current_frame_kernel, dim3(B), dim3(256), 0, stream, cur_frame, h, out, B, HW);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
