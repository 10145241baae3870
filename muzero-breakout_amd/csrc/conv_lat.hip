// Latent-resolution conv for the dynamics / prediction towers (bf16, gfx950 MFMA).
//
// The towers run 3x3 256->256 convs on a 4x5 latent (src/networks.py:19-35, 103-241):
// per env only 20 pixels x 256 channels (10 KB bf16), so a generic implicit GEMM re-reads
// every activation row once per tap and per column tile. Here a workgroup owns E whole
// envs (E*HW <= 160 rows, zero padding never crosses an env) and:
//   * loads those envs' input activations into LDS ONCE (16-B chunks XOR-swizzled by
//     row so the 32 rows of a fragment hit distinct banks) plus one zero row; every tap's
//     A fragment is a shifted LDS read (out-of-bounds taps read the zero row);
//   * streams the weights straight into VGPRs, each wave its own 32 output channels, from
//     a fragment-major packing Wf[col tile][half][k step][lane][8] (one fully coalesced 1 KB
//     wave load per 16-deep k step) with a register ring D steps deep; the buffer carries
//     8 extra k steps (8 KB) so the ring's loads are unconditional;
//   * computes 32x32 output tiles with v_mfma_f32_32x32x16_bf16, R = 5 row tiles per wave
//     (independent accumulation chains); 8 waves = 4 column tiles (128 output channels) x 2
//     channel halves of every tap (two waves per SIMD), halves summed through LDS;
//   * fused epilogue: + bias (BN folded) (+ per-(pixel, action) bias) (+ residual), ReLU.
// Grid: ceil(B/E) x ceil(Cout/128). At B = 1024: 128 x 2 = 256 workgroups = one per CU.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int R = 5;          // 32-row tiles per workgroup (E*HW <= 160)
constexpr int MAXROWS = 32 * R;

struct LatArgs {
  const bf16_t* in;
  long long in_env_stride;
  const int32_t* slot;
  long long in_slot_stride;
  const bf16_t* wf;       // [Cout/32][K/16][64][8]
  const float* bias;      // [Cout]
  const float* act_bias;  // optional [HW][A][Cout]
  const int32_t* act;     // [B]
  int A;
  const bf16_t* res;      // optional [B*HW][Cout]
  bf16_t* out;            // [B*HW][Cout]
  int B, H, W, Cin, Cout, ks, relu, E;
};

template <int KS, int CIN>
__global__ __launch_bounds__(512, 2) void conv_lat_kernel(LatArgs a) {
  constexpr int NC = CIN / 16;           // k steps per tap
  constexpr int NH = NC / 2;             // k steps per tap per wave (channel half)
  constexpr int NSW = KS * KS * NH;      // k steps per wave
  constexpr int D = NH >= 8 ? 8 : NH;    // weight ring depth (k steps in flight)
  constexpr int ROWB = CIN * 2;          // bytes per LDS row
  constexpr int NCHUNK = CIN / 8;        // 16-B chunks per row
  constexpr int SMASK = NCHUNK >= 16 ? 15 : NCHUNK - 1;
  constexpr int PAD = KS / 2;
  constexpr int NT = 512;
  static_assert(NH % D == 0, "ring / tap alignment");
  constexpr int LDS_A = (MAXROWS + 1) * ROWB, LDS_C = MAXROWS * 128 * 4;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_A > LDS_C ? LDS_A : LDS_C];
  __shared__ long long envoff[32 * R];
  const int HW = a.H * a.W;
  const int env0 = blockIdx.x * a.E;
  const int nenv = min(a.E, a.B - env0);
  const int rows = nenv * HW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wq = wave & 3, kh = wave >> 2;  // 32-column slot, channel half
  const int ct = blockIdx.y * 4 + wq;        // this wave's 32-column tile
  const bool active = ct * 32 < a.Cout;
  // weight stream first (latency hides under the staging); wf[ct][kh][step][lane][8] is
  // contiguous per wave and padded by 8 steps, so every ring load is unconditional.
  const uint4* wp = reinterpret_cast<const uint4*>(a.wf) + ((size_t)(active ? ct : 0) * 2 + kh) * NSW * 64 + lane;
  uint4 bq[D];
#pragma unroll
  for (int i = 0; i < D; ++i) bq[i] = wp[(size_t)i * 64];

  // per-env source base (slot gather resolved once, so the staging loads are branch-free)
  if (tid < a.E) {
    const int b = env0 + (tid < nenv ? tid : 0);
    long long off = (long long)b * a.in_env_stride;
    if (a.slot) off += (long long)a.slot[b] * a.in_slot_stride;
    envoff[tid] = off;
  }
  __syncthreads();
  // ---- stage the block's input activations (and the zero row) into LDS
  constexpr int TOTAL = (MAXROWS + 1) * NCHUNK;
  constexpr int PER = (TOTAL + NT - 1) / NT;
  {
    uint4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = u * NT + tid;
      const int r = i / NCHUNK, c = i % NCHUNK;
      const bool ok = i < TOTAL && r < rows;
      const int rr = ok ? r : 0;
      const int e = rr / HW, p = rr - (rr / HW) * HW;
      v[u] = *reinterpret_cast<const uint4*>(a.in + envoff[e] + (long long)p * CIN + c * 8);
      if (!ok) v[u] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = u * NT + tid;
      if (i < TOTAL) {
        const int r = i / NCHUNK, c = i % NCHUNK;
        *reinterpret_cast<uint4*>(lds + r * ROWB + ((c ^ (r & SMASK)) << 4)) = v[u];
      }
    }
  }
  __syncthreads();

  const int l32 = lane & 31, h = lane >> 5;
  f32x16 acc[R];
#pragma unroll
  for (int rt = 0; rt < R; ++rt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[rt][i] = 0.f;
  if (active) {
    int ry[R], rx[R], rbase[R];
    bool rval[R];
#pragma unroll
    for (int rt = 0; rt < R; ++rt) {
      const int m = rt * 32 + l32;
      rval[rt] = m < rows;
      const int e = m / HW, p = m - (m / HW) * HW;
      ry[rt] = p / a.W;
      rx[rt] = p - ry[rt] * a.W;
      rbase[rt] = e * HW;
    }
    // LDS byte offset of this lane's source row for tap t, and its chunk swizzle (<< 4)
    auto tap_rows = [&](int tap, int (&off)[R], int (&sw)[R]) {
      const int ky = tap / KS - PAD, kx = tap % KS - PAD;
#pragma unroll
      for (int rt = 0; rt < R; ++rt) {
        const int sy = ry[rt] + ky, sx = rx[rt] + kx;
        const bool ok = rval[rt] && sy >= 0 && sy < a.H && sx >= 0 && sx < a.W;
        const int r = ok ? rbase[rt] + sy * a.W + sx : MAXROWS;
        off[rt] = r * ROWB;
        sw[rt] = (r & SMASK) << 4;
      }
    };
    const int cbase = kh * NC + h;  // 16-B chunk of this lane's 8 channels at step 0 of a tap
    int offc[R], swc[R], offn[R], swn[R];
    tap_rows(0, offc, swc);
    bf16x8 afc[R], afn[R];
#pragma unroll
    for (int rt = 0; rt < R; ++rt)
      afc[rt] = *reinterpret_cast<const bf16x8*>(lds + offc[rt] + ((cbase << 4) ^ swc[rt]));
    for (int tap = 0; tap < KS * KS; ++tap) {
      if (tap + 1 < KS * KS) tap_rows(tap + 1, offn, swn);
#pragma unroll
      for (int c = 0; c < NH; ++c) {
        const int s = tap * NH + c;
        const uint4 bcur = bq[c % D];
        bq[c % D] = wp[(size_t)(s + D) * 64];
        // prefetch the next k step's A fragments (the next tap's rows after the last step)
        if (c + 1 < NH) {
          const int cb = (cbase + 2 * (c + 1)) << 4;
#pragma unroll
          for (int rt = 0; rt < R; ++rt) afn[rt] = *reinterpret_cast<const bf16x8*>(lds + offc[rt] + (cb ^ swc[rt]));
        } else if (tap + 1 < KS * KS) {
#pragma unroll
          for (int rt = 0; rt < R; ++rt)
            afn[rt] = *reinterpret_cast<const bf16x8*>(lds + offn[rt] + ((cbase << 4) ^ swn[rt]));
        }
        // pin the order: next-step reads + weight load in flight while this step's MFMAs run
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, bcur);
#pragma unroll
        for (int rt = 0; rt < R; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[rt], bfr, acc[rt], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 0; rt < R; ++rt) afc[rt] = afn[rt];
      }
#pragma unroll
      for (int rt = 0; rt < R; ++rt) { offc[rt] = offn[rt]; swc[rt] = swn[rt]; }
    }
  }

  // ---- epilogue, staged through LDS: channel-half 0 writes its f32 partial tile, half 1
  // adds its own (each element owned by one lane), then every lane finishes 16-B chunks:
  // + bias (+ act bias) (+ residual, 16-B loads), ReLU, bf16, 16-B stores.
  __syncthreads();  // every wave is done reading the A tile
  float* ot = reinterpret_cast<float*>(lds);
  if (active && kh == 0) {
#pragma unroll
    for (int rt = 0; rt < R; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) ot[(rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 128 + wq * 32 + l32] = acc[rt][r];
  }
  __syncthreads();
  if (active && kh == 1) {
#pragma unroll
    for (int rt = 0; rt < R; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float* p = ot + (rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 128 + wq * 32 + l32;
        *p = *p + acc[rt][r];
      }
  }
  __syncthreads();
  const int ncols = min(128, a.Cout - blockIdx.y * 128);
  const int ncb = ncols / 8;  // 16-B chunks per output row
  const int nchunks = rows * ncb;
  constexpr int EPT = (MAXROWS * 16 + NT - 1) / NT;  // chunks per thread (upper bound)
  uint4 rv[EPT];
  if (a.res) {
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      int i = u * NT + tid;
      i = i < nchunks ? i : 0;
      const int row = i / ncb, cc = i - (i / ncb) * ncb;
      const long long m = (long long)env0 * HW + row;
      rv[u] = *reinterpret_cast<const uint4*>(a.res + m * a.Cout + blockIdx.y * 128 + cc * 8);
    }
  }
#pragma unroll
  for (int u = 0; u < EPT; ++u) {
    const int i = u * NT + tid;
    if (i >= nchunks) break;
    const int row = i / ncb, cc = i - (i / ncb) * ncb;
    const long long m = (long long)env0 * HW + row;
    const int n0 = blockIdx.y * 128 + cc * 8;
    float v[8];
    const float4 x0 = *reinterpret_cast<const float4*>(ot + row * 128 + cc * 8);
    const float4 x1 = *reinterpret_cast<const float4*>(ot + row * 128 + cc * 8 + 4);
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    if (a.act_bias) {
      const int e = row / HW, p = row - e * HW;
      const float* ab = a.act_bias + ((long long)p * a.A + a.act[env0 + e]) * a.Cout + n0;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] + ab[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] + a.bias[n0 + j];
    if (a.res) {
      const uint32_t w[4] = {rv[u].x, rv[u].y, rv[u].z, rv[u].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] + bf16_to_f32((bf16_t)(w[j >> 1] >> (16 * (j & 1))));
    }
    if (a.relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    uint4 o;
    o.x = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
    o.y = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
    o.z = (uint32_t)f32_to_bf16(v[4]) | ((uint32_t)f32_to_bf16(v[5]) << 16);
    o.w = (uint32_t)f32_to_bf16(v[6]) | ((uint32_t)f32_to_bf16(v[7]) << 16);
    *reinterpret_cast<uint4*>(a.out + m * a.Cout + n0) = o;
  }
}

}  // namespace

extern "C" {

int mzba_conv_lat_supported(int H, int W, int Cin, int Cout, int ks) {
  const int HW = H * W;
  if (HW > 32 * R || HW <= 0) return 0;
  if (!(Cin == 64 || Cin == 128 || Cin == 256) || Cout % 32 != 0) return 0;
  if (!(ks == 1 || ks == 3)) return 0;
  return 1;
}

int mzba_conv_lat(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                  const void* wf, const float* bias, const float* act_bias, const int32_t* act, int A,
                  const void* res, void* out, int B, int H, int W, int Cin, int Cout, int ks, int relu,
                  hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && mzba_conv_lat_supported(H, W, Cin, Cout, ks), -1);
  MZ_CHECK_ARG(!act_bias || (act && A > 0), -3);
  const int HW = H * W;
  const int E = (32 * R) / HW;
  LatArgs a{(const bf16_t*)in, in_env_stride, slot, in_slot_stride, (const bf16_t*)wf, bias, act_bias, act, A,
            (const bf16_t*)res, (bf16_t*)out, B, H, W, Cin, Cout, ks, relu, E};
  dim3 grid((B + E - 1) / E, (Cout + 127) / 128);
#define MZ_LAT(KS_, CIN_) \
  if (ks == KS_ && Cin == CIN_) { hipLaunchKernelGGL((conv_lat_kernel<KS_, CIN_>), grid, dim3(512), 0, stream, a); }
  MZ_LAT(3, 256) else MZ_LAT(1, 256) else MZ_LAT(3, 128) else MZ_LAT(1, 128) else MZ_LAT(3, 64) else MZ_LAT(1, 64)
#undef MZ_LAT
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
