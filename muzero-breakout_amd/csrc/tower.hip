// Fused residual tower for the dynamics / prediction nets (bf16, gfx950 MFMA).
//
// The towers are nblocks x ResidualBlock(256) on a 4x5 latent (src/networks.py:19-35,
// 124-131, 190-197). Launching every conv separately re-stages the activations into LDS
// and writes them back to HBM 28 times per tower. Here ONE workgroup owns E = 4 whole envs
// (80 rows) x all 256 channels for the whole tower:
//   * X (block input / output) and T (conv1 output) stay resident in LDS (2 x 40 KB,
//     16-B chunks XOR-swizzled by row) across every block; one zero row serves the padding;
//   * weights stream into VGPRs from a 16-column fragment-major packing
//     wf16[col tile][k step][lane][8] (one coalesced 1 KB wave load per 32-deep k step and
//     column tile, 8 steps in flight); each of the 8 waves owns 32 output channels;
//   * v_mfma_f32_16x16x32_bf16: 5 row tiles x 2 column tiles per wave = 10 independent
//     accumulators; MFMA / next-step ds_read_b128 / VALU interleaved by sched_group_barrier;
//   * conv1 epilogue: + bias, ReLU -> T (LDS); conv2: accumulator initialised with
//     bias + residual X, ReLU -> X in place (each element is owned by one lane).
// Input is read from HBM once (optional per-env slot gather from the latent node pool) and
// the tower output written once. Grid: ceil(B / 4) workgroups of 512 threads.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int TE = 4;              // envs per workgroup
constexpr int TROWS = 80;          // TE * 20 (4x5 latent)
constexpr int TC = 256;            // channels
constexpr int TROWB = TC * 2;      // 512 B per LDS row
constexpr int TR = 5;              // 16-row tiles
constexpr int TNS = 9 * TC / 32;   // 72 k steps per 3x3 conv
constexpr int TD = 4;              // weight ring depth (k steps)
constexpr int TNT = 512;

struct TowerArgs {
  const bf16_t* in;
  long long in_env_stride;
  const int32_t* slot;
  long long in_slot_stride;
  bf16_t* out;               // [B][20][256]
  const bf16_t* wf;          // per conv: [16 col tiles][72 k steps][64][8], convs back to back (+pad)
  const float* bias;         // per conv: [256]
  int nblocks;               // residual blocks (2 convs each)
  int B;
};

// LDS byte offset of (row, 16-B chunk) in a swizzled activation image
MZ_DEV int toff(int row, int chunk) { return row * TROWB + ((chunk ^ (row & 15)) << 4); }

template <bool RESID>
__device__ __forceinline__ void tower_conv(const TowerArgs& a, const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                           const uint4* __restrict__ wconv, const float* __restrict__ bconv,
                                           const int (&ry)[TR], const int (&rx)[TR], const int (&rb)[TR],
                                           const bool (&rv)[TR], int lane, int wave) {
  const int q = lane >> 4, l16 = lane & 15;
  const int ct0 = 2 * wave, ct1 = 2 * wave + 1;  // 16-column tiles of this wave
  const uint4* wp0 = wconv + (size_t)ct0 * TNS * 64 + lane;
  const uint4* wp1 = wconv + (size_t)ct1 * TNS * 64 + lane;
  uint4 b0q[TD], b1q[TD];
#pragma unroll
  for (int i = 0; i < TD; ++i) { b0q[i] = wp0[(size_t)i * 64]; b1q[i] = wp1[(size_t)i * 64]; }
  // accumulator init: bias (+ residual X for conv2); D[row = 4q + i][col = l16]
  const int n0 = ct0 * 16 + l16, n1 = ct1 * 16 + l16;
  const float bb0 = bconv[n0], bb1 = bconv[n1];
  f32x4 acc0[TR], acc1[TR];
#pragma unroll
  for (int rt = 0; rt < TR; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float r0 = bb0, r1 = bb1;
      if (RESID) {
        const int row = rt * 16 + 4 * q + i;
        const bf16_t* xr = reinterpret_cast<const bf16_t*>(dst + toff(row, n0 >> 3)) + (n0 & 7);
        const bf16_t* xr1 = reinterpret_cast<const bf16_t*>(dst + toff(row, n1 >> 3)) + (n1 & 7);
        r0 = r0 + bf16_to_f32(*xr);
        r1 = r1 + bf16_to_f32(*xr1);
      }
      acc0[rt][i] = r0;
      acc1[rt][i] = r1;
    }
  auto tap_rows = [&](int tap, int (&off)[TR], int (&sw)[TR]) {
    const int ky = tap / 3 - 1, kx = tap % 3 - 1;
#pragma unroll
    for (int rt = 0; rt < TR; ++rt) {
      const int sy = ry[rt] + ky, sx = rx[rt] + kx;
      const bool ok = rv[rt] && sy >= 0 && sy < 4 && sx >= 0 && sx < 5;
      const int r = ok ? rb[rt] + sy * 5 + sx : TROWS;
      off[rt] = r * TROWB;
      sw[rt] = (r & 15) << 4;
    }
  };
  int offc[TR], swc[TR], offn[TR], swn[TR];
  tap_rows(0, offc, swc);
  bf16x8 afc[TR], afn[TR];
#pragma unroll
  for (int rt = 0; rt < TR; ++rt) afc[rt] = *reinterpret_cast<const bf16x8*>(src + offc[rt] + ((q << 4) ^ swc[rt]));
  constexpr int NC = TC / 32;  // 8 k steps per tap
  for (int tap = 0; tap < 9; ++tap) {
    tap_rows(tap < 8 ? tap + 1 : tap, offn, swn);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int s = tap * NC + c;
      const bf16x8 w0 = __builtin_bit_cast(bf16x8, b0q[c % TD]);
      const bf16x8 w1 = __builtin_bit_cast(bf16x8, b1q[c % TD]);
      b0q[c % TD] = wp0[(size_t)(s + TD) * 64];
      b1q[c % TD] = wp1[(size_t)(s + TD) * 64];
#pragma unroll
      for (int rt = 0; rt < TR; ++rt) {
        acc0[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afc[rt], w0, acc0[rt], 0, 0, 0);
        acc1[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afc[rt], w1, acc1[rt], 0, 0, 0);
        if (c + 1 < NC)
          afn[rt] = *reinterpret_cast<const bf16x8*>(src + offc[rt] + (((4 * (c + 1) + q) << 4) ^ swc[rt]));
        else
          afn[rt] = *reinterpret_cast<const bf16x8*>(src + offn[rt] + ((q << 4) ^ swn[rt]));
      }
#pragma unroll
      for (int rt = 0; rt < TR; ++rt) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rt = 0; rt < TR; ++rt) afc[rt] = afn[rt];
    }
#pragma unroll
    for (int rt = 0; rt < TR; ++rt) { offc[rt] = offn[rt]; swc[rt] = swn[rt]; }
  }
  // epilogue: ReLU -> bf16 -> dst (T for conv1, X in place for conv2)
#pragma unroll
  for (int rt = 0; rt < TR; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rt * 16 + 4 * q + i;
      *(reinterpret_cast<bf16_t*>(dst + toff(row, n0 >> 3)) + (n0 & 7)) = f32_to_bf16(fmaxf(acc0[rt][i], 0.f));
      *(reinterpret_cast<bf16_t*>(dst + toff(row, n1 >> 3)) + (n1 & 7)) = f32_to_bf16(fmaxf(acc1[rt][i], 0.f));
    }
}

__global__ __launch_bounds__(TNT, 2) void tower_kernel(TowerArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[(TROWS + 1) * TROWB];  // X + zero row
  __shared__ __attribute__((aligned(16))) uint8_t ts[(TROWS + 1) * TROWB];  // T + zero row
  __shared__ long long envoff[TE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int env0 = blockIdx.x * TE;
  const int nenv = min(TE, a.B - env0);
  const int rows = nenv * 20;
  if (tid < TE) {
    const int b = env0 + (tid < nenv ? tid : 0);
    long long off = (long long)b * a.in_env_stride;
    if (a.slot) off += (long long)a.slot[b] * a.in_slot_stride;
    envoff[tid] = off;
  }
  __syncthreads();
  // stage X (80 rows x 32 chunks = 2560 chunks, 5 per thread) and zero both pad rows
  {
    uint4 v[5];
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int i = u * TNT + tid;
      const int r = i >> 5, c = i & 31;
      const bool ok = r < rows;
      const int rr = ok ? r : 0;
      v[u] = *reinterpret_cast<const uint4*>(a.in + envoff[rr / 20] + (long long)(rr % 20) * TC + c * 8);
      if (!ok) v[u] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int i = u * TNT + tid;
      *reinterpret_cast<uint4*>(xs + toff(i >> 5, i & 31)) = v[u];
    }
    if (tid < 32) {
      *reinterpret_cast<uint4*>(xs + TROWS * TROWB + tid * 16) = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(ts + TROWS * TROWB + tid * 16) = make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();
  // per row tile: this lane's A row geometry (row = rt*16 + (lane & 15))
  int ry[TR], rx[TR], rb[TR];
  bool rv[TR];
#pragma unroll
  for (int rt = 0; rt < TR; ++rt) {
    const int m = rt * 16 + (lane & 15);
    rv[rt] = m < rows;
    const int e = m / 20, p = m - e * 20;
    ry[rt] = p / 5; rx[rt] = p - (p / 5) * 5; rb[rt] = e * 20;
  }
  const uint4* wf = reinterpret_cast<const uint4*>(a.wf);
  constexpr size_t WCONV = (size_t)16 * TNS * 64;  // uint4 per conv
  for (int blk = 0; blk < a.nblocks; ++blk) {
    tower_conv<false>(a, xs, ts, wf + (2 * blk) * WCONV, a.bias + (2 * blk) * TC, ry, rx, rb, rv, lane, wave);
    __syncthreads();
    tower_conv<true>(a, ts, xs, wf + (2 * blk + 1) * WCONV, a.bias + (2 * blk + 1) * TC, ry, rx, rb, rv, lane, wave);
    __syncthreads();
  }
  // write the tower output (16-B chunks, rows < rows)
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int i = u * TNT + tid;
    const int r = i >> 5, c = i & 31;
    if (r < rows)
      *reinterpret_cast<uint4*>(a.out + (long long)(env0 + r / 20) * 20 * TC + (r % 20) * TC + c * 8) =
          *reinterpret_cast<const uint4*>(xs + toff(r, c));
  }
}

}  // namespace

extern "C" {

// nblocks residual blocks (256 ch, 4x5) fused; wf16: per conv [16][72][64][8] bf16 (+8 KB pad after
// the last conv), bias: per conv [256] f32 (BN folded). in: env b at in + b*in_env_stride
// (+ slot[b]*in_slot_stride); out: [B][20][256].
int mzba_tower(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride, void* out,
               const void* wf16, const float* bias, int nblocks, int B, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nblocks >= 1 && in && out && wf16 && bias, -1);
  TowerArgs a{(const bf16_t*)in, in_env_stride, slot, in_slot_stride, (bf16_t*)out, (const bf16_t*)wf16, bias,
              nblocks, B};
  hipLaunchKernelGGL(tower_kernel, dim3((B + TE - 1) / TE), dim3(TNT), 0, stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
