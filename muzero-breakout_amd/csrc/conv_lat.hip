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

#ifdef MZ_LAT_STAMPS
// diagnostic build only (libmzba_diag.so, tools/stamp_conv.py): per-workgroup phase stamps
__device__ unsigned long long mz_lat_stamps[4096][8];
#define MZ_STAMP(k)                                                                        \
  do {                                                                                     \
    if ((threadIdx.x & 63) == 0 && blockIdx.x + gridDim.x * blockIdx.y < 4096) {           \
      const int w_ = threadIdx.x >> 6;                                                     \
      if (w_ == 0 || (k == 3 && w_ == 4))                                                  \
        mz_lat_stamps[blockIdx.x + gridDim.x * blockIdx.y][(k == 3 && w_ == 4) ? 7 : k] =  \
            __builtin_amdgcn_s_memtime();                                                  \
    }                                                                                      \
  } while (0)
#else
#define MZ_STAMP(k) do {} while (0)
#endif
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
  // learner: the consuming BatchNorm's batch statistics in the epilogue (mzba_conv_lat_bn), per
  // workgroup (chunk = blockIdx.x, its rows): smode 1: part[chunk][n] = (mean, M2) of the bf16
  // outputs; smode 2: the output becomes g = out * [sy > 0] and part[chunk][n] = (sum g,
  // sum g (sx - smean[n])) — bn_stats_partial / bn_bwd_partial (learn.hip) without their launches
  int smode;
  float2* part;
  const bf16_t* sy;
  const bf16_t* sx;
  const float* smean;
  // learner: the producing BatchNorm's apply in the staging (pstats != null): the staged input is
  // y = [prelu](in * alpha + beta' [+ pres]) with alpha / beta' = pstats rows 2 / 3, and the
  // workgroups of column block 0 also store y to pout (the BN output the backward needs)
  const float* pstats;
  const bf16_t* pres;
  int prelu;
  bf16_t* pout;
  // backward (pcoef != null): the staged input is the BN input gradient dt = ((g - (x - mean) k) -
  // mean_g) alpha of the BN output gradient g = in and BN input x = pres (mean / alpha = pstats rows
  // 0 / 2, mean_g / k = pcoef rows 0 / 1: mzba_bn_backward_coef), also stored to pout
  const float* pcoef;
  // learner: the consuming BatchNorm's finaliser in this launch (ctr != null, smode 1 / 2; lat_bn_finish): the last
  // workgroup of each column block folds every workgroup's partials. smode 1: fstats = out [4][Cout] (mean, invstd,
  // alpha, beta'), running statistics updated in place (optional); smode 2: fstats = in (invstd row 1, alpha row 2),
  // dgamma / dbeta += in place, coef = out [3][Cout] (mean_g, k, alpha) — bn_stats_final_kernel /
  // bn_bwd_final_kernel (learn.hip) without their launches
  unsigned* ctr;  // [Cout / 128] zero at entry; the last workgroup of a column block resets its word
  float eps, momentum;
  const float* gamma;
  const float* beta;
  float* fstats;
  float* run_mean;
  float* run_var;
  float* dgamma;
  float* dbeta;
  float* coef;
};

// The consuming BatchNorm's finaliser at the end of the producing launch. Every workgroup has stored its partials
// with sc1 stores (lat_epilogue); after every wave's stores have completed (vmcnt(0), then a workgroup barrier) one
// lane adds to its column block's counter, and the workgroup whose add returns gridDim.x - 1 loads all the
// partials with sc1 loads — the hand-off of MI355X_MICROARCH.md's table, row 1 (one workgroup per CU: conv_lat's
// 8-wave instances hold > 80 KiB of LDS; hipMalloc memory) — and folds them, 4 threads per channel (chunks
// q, q + 4, ...) combined in q order: forward mean = sum n_k mean_k / M, M2 = sum (M2_k + n_k (mean_k - mean)^2)
// in double (the division-free fold of the chunk statistics), backward sum g and sum g (x - mean) in double; then
// the tails of bn_stats_final_kernel / bn_bwd_final_kernel, expression for expression. The fold order differs
// from those kernels' (Chan pairs + butterfly), so statistics can differ from theirs in the last f32 place.
template <int NT>
__device__ __forceinline__ void lat_bn_finish(const LatArgs& a, float* ws, int tid) {
  static_assert(NT == 512, "4 threads per channel of a 128-channel column block");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have completed
  __syncthreads();
  volatile int* flag = reinterpret_cast<volatile int*>(ws);
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.ctr + blockIdx.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == gridDim.x - 1;
    if (last) __hip_atomic_store(a.ctr + blockIdx.y, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  const int col = tid & 127, q = tid >> 7;
  const int n = blockIdx.y * 128 + col;
  const int nchunk = gridDim.x, rpc = a.E * a.H * a.W, M = a.B * a.H * a.W;
  unsigned long long* P = reinterpret_cast<unsigned long long*>(a.part) + n;  // float2 [chunk][Cout]
  auto ld = [&](int k) {
    const unsigned long long u = __hip_atomic_load(P + (size_t)k * a.Cout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float2(__uint_as_float((unsigned)u), __uint_as_float((unsigned)(u >> 32)));
  };
  auto nk = [&](int k) { return (double)min(rpc, M - k * rpc); };
  constexpr int CK = 16;  // chunks per thread held in registers (nchunk <= 64: all of them)
  float2 pv[CK];
#pragma unroll
  for (int i = 0; i < CK; ++i) pv[i] = q + 4 * i < nchunk ? ld(q + 4 * i) : make_float2(0.f, 0.f);
  double* rd = reinterpret_cast<double*>(ws) + 8;  // [4][128] after the flag
  auto fold4 = [&](double v) {  // (v_0 + v_1) + v_2 + v_3 over q, every thread gets it
    __syncthreads();
    rd[q * 128 + col] = v;
    __syncthreads();
    return ((rd[col] + rd[128 + col]) + rd[256 + col]) + rd[384 + col];
  };
  if (a.smode == 1) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < CK; ++i)
      if (q + 4 * i < nchunk) s += nk(q + 4 * i) * (double)pv[i].x;
    for (int k = q + 4 * CK; k < nchunk; k += 4) s += nk(k) * (double)ld(k).x;
    const double mean = fold4(s) / M;
    double m2 = 0;
#pragma unroll
    for (int i = 0; i < CK; ++i)
      if (q + 4 * i < nchunk) {
        const double d = (double)pv[i].x - mean;
        m2 += (double)pv[i].y + nk(q + 4 * i) * d * d;
      }
    for (int k = q + 4 * CK; k < nchunk; k += 4) {
      const float2 v = ld(k);
      const double d = (double)v.x - mean;
      m2 += (double)v.y + nk(k) * d * d;
    }
    m2 = fold4(m2);
    if (q) return;
    const int C = a.Cout;
    const float var = (float)(m2 / M);
    const float invstd = (float)(1.0 / sqrt((double)var + (double)a.eps));
    const float alpha = invstd * a.gamma[n];
    const float fm = (float)mean;
    a.fstats[n] = fm;
    a.fstats[C + n] = invstd;
    a.fstats[2 * C + n] = alpha;
    a.fstats[3 * C + n] = a.beta[n] - fm * alpha;
    if (a.run_mean) {
      a.run_mean[n] = (float)((double)a.momentum * mean + (1.0 - (double)a.momentum) * (double)a.run_mean[n]);
      const double unbiased = M > 1 ? m2 / (double)(M - 1) : m2;
      a.run_var[n] = (float)((double)a.momentum * unbiased + (1.0 - (double)a.momentum) * (double)a.run_var[n]);
    }
    return;
  }
  double sg = 0, dot = 0;
#pragma unroll
  for (int i = 0; i < CK; ++i) {
    sg += (double)pv[i].x;  // chunks past nchunk hold exact zeros
    dot += (double)pv[i].y;
  }
  for (int k = q + 4 * CK; k < nchunk; k += 4) {
    const float2 v = ld(k);
    sg += (double)v.x;
    dot += (double)v.y;
  }
  sg = fold4(sg);
  dot = fold4(dot);
  if (q) return;
  const int C = a.Cout;
  const float invstd = a.fstats[C + n], alpha = a.fstats[2 * C + n];
  a.dgamma[n] = a.dgamma[n] + (float)dot * invstd;
  a.dbeta[n] = a.dbeta[n] + (float)sg;
  a.coef[n] = (float)(sg / M);
  a.coef[C + n] = (float)dot * invstd * invstd / (float)M;
  a.coef[2 * C + n] = alpha;
}

// epilogue: (1) issue the residual loads (16 B per lane) so they land while the f32 tile is
// reduced through LDS; (2) finish 16-B output chunks: + residual, ReLU, bf16, 16-B stores.
// Bias and the per-(pixel, action) bias were folded into the accumulator init.
constexpr int EPT_MAX = 10;
template <int NT, int MR = MAXROWS>
__device__ __forceinline__ void lat_res_prefetch(const LatArgs& a, uint4 (&rv)[EPT_MAX], int rows, int env0, int HW,
                                                 int tid) {
  constexpr int EPT = (MR * 16 + NT - 1) / NT;
  // int arithmetic (min(int, unsigned) resolved to the double overload: a v_min_f64 round trip per call)
  const int ncols = min(128, a.Cout - (int)blockIdx.y * 128);
  const int ncb = ncols / 8;
  const int nchunks = rows * ncb;
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
}
template <int NT, int MR = MAXROWS>
__device__ __forceinline__ void lat_epilogue(const LatArgs& a, float* ot, const uint4 (&rv)[EPT_MAX], int rows,
                                             int env0, int HW, int tid) {
  constexpr int EPT = (MR * 16 + NT - 1) / NT;
  const int ncols = min(128, a.Cout - (int)blockIdx.y * 128);
  const int ncb = ncols / 8;
  const int nchunks = rows * ncb;
  // smode 2: this thread's chunk column is fixed (ncb = 16 divides NT): register partial sums
  float sg[8], sd[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sg[j] = 0.f; sd[j] = 0.f; mu[j] = 0.f; }
  if (a.smode == 2) {
    const int n0 = blockIdx.y * 128 + (tid % ncb) * 8;
    const float4 m0 = *reinterpret_cast<const float4*>(a.smean + n0), m1 = *reinterpret_cast<const float4*>(a.smean + n0 + 4);
    mu[0] = m0.x; mu[1] = m0.y; mu[2] = m0.z; mu[3] = m0.w; mu[4] = m1.x; mu[5] = m1.y; mu[6] = m1.z; mu[7] = m1.w;
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
    if (a.smode == 1) {  // the stored (bf16-rounded) values back into the tile for the column pass
      const uint32_t w[4] = {o.x, o.y, o.z, o.w};
      float r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = bf16_to_f32((bf16_t)(w[j >> 1] >> (16 * (j & 1))));
      *reinterpret_cast<float4*>(ot + row * 128 + cc * 8) = make_float4(r[0], r[1], r[2], r[3]);
      *reinterpret_cast<float4*>(ot + row * 128 + cc * 8 + 4) = make_float4(r[4], r[5], r[6], r[7]);
    } else if (a.smode == 2) {  // ReLU mask of the BN output, masked g stored, partial sums
      const uint4 yv = *reinterpret_cast<const uint4*>(a.sy + m * a.Cout + n0);
      const uint4 xv = *reinterpret_cast<const uint4*>(a.sx + m * a.Cout + n0);
      const uint32_t w[4] = {o.x, o.y, o.z, o.w}, yw[4] = {yv.x, yv.y, yv.z, yv.w}, xw[4] = {xv.x, xv.y, xv.z, xv.w};
      uint32_t ow[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int sh = 16 * (j & 1);
        const bool keep = bf16_to_f32((bf16_t)(yw[j >> 1] >> sh)) > 0.f;
        const uint32_t gb = keep ? ((w[j >> 1] >> sh) & 0xffffu) : 0u;
        ow[j >> 1] |= gb << sh;
        const float g = bf16_to_f32((bf16_t)gb);
        sg[j] += g;
        sd[j] += g * (bf16_to_f32((bf16_t)(xw[j >> 1] >> sh)) - mu[j]);
      }
      o = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    }
    *reinterpret_cast<uint4*>(a.out + m * a.Cout + n0) = o;
  }
  if (a.smode == 0) return;
  __syncthreads();  // the tile holds the rounded outputs (1) / every thread is done with it (2)
  float* pf = reinterpret_cast<float*>(a.part) + 2 * ((size_t)blockIdx.x * a.Cout + blockIdx.y * 128);
  if (a.smode == 1) {  // (mean, M2) per column over the rows: NT / 128 row groups, lanes = columns
    constexpr int TPC = NT / 128;  // (a wave reads 64 consecutive columns of one row: conflict-free)
    const int col = tid % 128, q = tid / 128;
    float* red = ot + MR * 128;    // [TPC][128] after the tile (LDS_C covers MR rows; see caller)
    // every row's value read before the first add (one LDS round trip, not one per row of a rolled loop);
    // rows past `rows` add an exact 0, so the sums are the rolled loop's, bit for bit
    constexpr int RPT = MR / TPC;
    float s = 0.f;
    if (col < ncols) {
      float vv[RPT];
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        const int r = q + k * TPC;
        vv[k] = r < rows ? ot[r * 128 + col] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < RPT; ++k) s += vv[k];
    }
    red[q * 128 + col] = s;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < TPC; ++k) tot += red[k * 128 + col];
    const float mean = tot / rows;
    float m2 = 0.f;
    if (col < ncols) {
      float vv[RPT];
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        const int r = q + k * TPC;
        vv[k] = r < rows ? ot[r * 128 + col] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        const float d = q + k * TPC < rows ? vv[k] - mean : 0.f;
        m2 += d * d;
      }
    }
    __syncthreads();
    red[q * 128 + col] = m2;
    __syncthreads();
    if (q == 0 && col < ncols) {
      float t2 = 0.f;
#pragma unroll
      for (int k = 0; k < TPC; ++k) t2 += red[k * 128 + col];
      if (a.ctr)  // one 8-B sc1 store (lat_bn_finish's hand-off)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(pf + 2 * col),
                           (unsigned long long)__float_as_uint(mean) | ((unsigned long long)__float_as_uint(t2) << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else {
        pf[2 * col] = mean;
        pf[2 * col + 1] = t2;
      }
    }
    if constexpr (NT == 512)
      if (a.ctr) lat_bn_finish<NT>(a, ot, tid);
    return;
  }
  // smode 2: the NT / ncb threads of a chunk column reduce through the tile, in thread order
  constexpr int G = NT / 16;
  float* rg = ot;              // [G][128]
  float* rd = ot + G * 128;    // [G][128]
  const int grp = tid / ncb, cc = tid % ncb;
#pragma unroll
  for (int j = 0; j < 8; ++j) { rg[grp * 128 + cc * 8 + j] = sg[j]; rd[grp * 128 + cc * 8 + j] = sd[j]; }
  __syncthreads();
  if (tid < 2 * 128) {
    const int col = tid & 127;
    const float* src = tid < 128 ? rg : rd;
    float t = 0.f;
    for (int k = 0; k < G; ++k) t += src[k * 128 + col];
    if (col < ncols) {
      if (a.ctr)  // sc1 store (lat_bn_finish's hand-off)
        __hip_atomic_store(reinterpret_cast<unsigned*>(pf + 2 * col + (tid >> 7)), __float_as_uint(t), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      else
        pf[2 * col + (tid >> 7)] = t;
    }
  }
  if constexpr (NT == 512)
    if (a.ctr) lat_bn_finish<NT>(a, ot, tid);
}

// accumulator init for the first channel group: bias (+ per-(pixel, action) bias) of this
// lane's (row, col) elements, so the epilogue only adds the residual.
__device__ __forceinline__ float lat_acc_init(const LatArgs& a, float bias_n, int row, int rows, int n, int env0,
                                              int HW) {
  float v = bias_n;
  if (a.act_bias) {
    const int rr = row < rows ? row : 0;
    const int e = rr / HW, p = rr - e * HW;
    v = a.act_bias[((long long)p * a.A + a.act[env0 + e]) * a.Cout + n] + v;
  }
  return v;
}

// RT: 32-row tiles per workgroup (5: E*HW <= 160; 3: E*HW <= 96, twice the workgroups for the
// learner's B = 512 latent convs, whose 5-tile grid fills only half the CUs)
// OCC: workgroups per CU the register budget allows (2: <= 128 VGPRs at 8 waves, the 3-row instance with a 4-deep
// ring whose ~56 KiB of LDS lets two workgroups share a CU, one's staging / epilogue beside the other's k loop)
template <int KS, int CIN, int WAVES, int DMAX, int RT = R, int OCC = 1>
__global__ __launch_bounds__(64 * WAVES, OCC * WAVES / 4) void conv_lat_kernel(LatArgs a) {
  constexpr int MAXROWS = 32 * RT;
  constexpr int KSPLIT = WAVES / 4;      // channel groups per tap (1: 4 waves, 2: 8 waves)
  constexpr int NC = CIN / 16;           // k steps per tap
  constexpr int NH = NC / KSPLIT;        // k steps per tap per wave
  constexpr int NSW = KS * KS * NH;      // k steps per wave
  constexpr int D = NH >= DMAX ? DMAX : NH;  // weight ring depth (k steps in flight)
  constexpr int ROWB = CIN * 2;          // bytes per LDS row
  constexpr int NCHUNK = CIN / 8;        // 16-B chunks per row
  constexpr int SMASK = NCHUNK >= 16 ? 15 : NCHUNK - 1;
  constexpr int PAD = KS / 2;
  constexpr int NT = 64 * WAVES;
  static_assert(NH % D == 0, "ring / tap alignment");
  constexpr int LDS_A = (MAXROWS + 1) * ROWB, LDS_C = (MAXROWS + NT / 128) * 128 * 4;  // + BN-stats scratch
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_A > LDS_C ? LDS_A : LDS_C];
  __shared__ long long envoff[32 * RT];
  __shared__ float s_ab[4][CIN];  // BN prologue: alpha, beta' (forward) / mean, alpha, mean_g, k (backward)
  const int HW = a.H * a.W;
  const int env0 = blockIdx.x * a.E;
  const int nenv = min(a.E, a.B - env0);
  const int rows = nenv * HW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wq = wave & 3, kh = wave >> 2;  // 32-column slot, channel group
  const int ct = blockIdx.y * 4 + wq;        // this wave's 32-column tile
  const bool active = ct * 32 < a.Cout;
  // weight stream first (latency hides under the staging); wf[ct][kh][step][lane][8] is
  // contiguous per wave and padded by 8 steps, so every ring load is unconditional.
  MZ_STAMP(0);
  const uint4* wp = reinterpret_cast<const uint4*>(a.wf) + ((size_t)(active ? ct : 0) * KSPLIT + kh) * NSW * 64 + lane;
  uint4 bq[D];
#pragma unroll
  for (int i = 0; i < D; ++i) bq[i] = wp[(size_t)i * 64];
  const float bias_n = a.bias[active ? ct * 32 + (lane & 31) : 0];  // lands during the staging

  // per-env source base (slot gather resolved once, so the staging loads are branch-free)
  if (tid < a.E) {
    const int b = env0 + (tid < nenv ? tid : 0);
    long long off = (long long)b * a.in_env_stride;
    if (a.slot) off += (long long)a.slot[b] * a.in_slot_stride;
    envoff[tid] = off;
  }
  if (a.pstats && !a.pcoef)
    for (int c = tid; c < CIN; c += NT) { s_ab[0][c] = a.pstats[2 * CIN + c]; s_ab[1][c] = a.pstats[3 * CIN + c]; }
  if (a.pcoef)
    for (int c = tid; c < CIN; c += NT) {
      s_ab[0][c] = a.pstats[c]; s_ab[1][c] = a.pstats[2 * CIN + c];
      s_ab[2][c] = a.pcoef[c]; s_ab[3][c] = a.pcoef[CIN + c];
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
    if (a.pstats) {  // BN apply (learner): rows are contiguous NHWC, env stride HW * CIN
      uint4 rv[PER];
      if (a.pres) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int i = u * NT + tid;
          const int r = i / NCHUNK, c = i % NCHUNK;
          const int rr = (i < TOTAL && r < rows) ? r : 0;
          rv[u] = *reinterpret_cast<const uint4*>(a.pres + ((long long)env0 * HW + rr) * CIN + c * 8);
        }
      }
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int i = u * NT + tid;
        const int r = i / NCHUNK, c = i % NCHUNK;
        if (!(i < TOTAL && r < rows)) continue;
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        uint32_t rw[4] = {0u, 0u, 0u, 0u};
        if (a.pres) { rw[0] = rv[u].x; rw[1] = rv[u].y; rw[2] = rv[u].z; rw[3] = rv[u].w; }
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ch = c * 8 + 2 * q;
          float y0, y1;
          if (a.pcoef) {  // bn_bwd_apply's expression, same op order
            const float g0 = bf16_to_f32((bf16_t)(w[q] & 0xffffu)), g1 = bf16_to_f32((bf16_t)(w[q] >> 16));
            const float x0 = bf16_to_f32((bf16_t)(rw[q] & 0xffffu)), x1 = bf16_to_f32((bf16_t)(rw[q] >> 16));
            y0 = ((g0 - (x0 - s_ab[0][ch]) * s_ab[3][ch]) - s_ab[2][ch]) * s_ab[1][ch];
            y1 = ((g1 - (x1 - s_ab[0][ch + 1]) * s_ab[3][ch + 1]) - s_ab[2][ch + 1]) * s_ab[1][ch + 1];
          } else {
            y0 = bf16_to_f32((bf16_t)(w[q] & 0xffffu)) * s_ab[0][ch] + s_ab[1][ch];
            y1 = bf16_to_f32((bf16_t)(w[q] >> 16)) * s_ab[0][ch + 1] + s_ab[1][ch + 1];
            if (a.pres) {
              y0 = y0 + bf16_to_f32((bf16_t)(rw[q] & 0xffffu));
              y1 = y1 + bf16_to_f32((bf16_t)(rw[q] >> 16));
            }
            if (a.prelu) { y0 = fmaxf(y0, 0.f); y1 = fmaxf(y1, 0.f); }
          }
          o[q] = (uint32_t)f32_to_bf16(y0) | ((uint32_t)f32_to_bf16(y1) << 16);
        }
        v[u] = make_uint4(o[0], o[1], o[2], o[3]);
        if (blockIdx.y == 0)
          *reinterpret_cast<uint4*>(a.pout + ((long long)env0 * HW + r) * CIN + c * 8) = v[u];
      }
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
  MZ_STAMP(1);

  const int l32 = lane & 31, h = lane >> 5;
  f32x16 acc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      acc[rt][i] = (active && kh == 0) ? lat_acc_init(a, bias_n, rt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h, rows,
                                                     ct * 32 + l32, env0, HW)
                                       : 0.f;
  if (active) {
    int ry[RT], rx[RT], rbase[RT];
    bool rval[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int m = rt * 32 + l32;
      rval[rt] = m < rows;
      const int e = m / HW, p = m - (m / HW) * HW;
      ry[rt] = p / a.W;
      rx[rt] = p - ry[rt] * a.W;
      rbase[rt] = e * HW;
    }
    // LDS byte offset of this lane's source row for tap t, and its chunk swizzle (<< 4)
    auto tap_rows = [&](int tap, int (&off)[RT], int (&sw)[RT]) {
      const int ky = tap / KS - PAD, kx = tap % KS - PAD;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int sy = ry[rt] + ky, sx = rx[rt] + kx;
        const bool ok = rval[rt] && sy >= 0 && sy < a.H && sx >= 0 && sx < a.W;
        const int r = ok ? rbase[rt] + sy * a.W + sx : MAXROWS;
        off[rt] = r * ROWB;
        sw[rt] = (r & SMASK) << 4;
      }
    };
    const int cbase = kh * (2 * NH) + h;  // 16-B chunk of this lane's 8 channels at step 0 of a tap
    int offc[RT], swc[RT], offn[RT], swn[RT];
    tap_rows(0, offc, swc);
    bf16x8 afc[RT], afn[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      afc[rt] = *reinterpret_cast<const bf16x8*>(lds + offc[rt] + ((cbase << 4) ^ swc[rt]));
    for (int tap = 0; tap < KS * KS; ++tap) {
      // next tap's source rows (the last tap re-reads its own rows: harmless, branch-free)
      tap_rows(tap + 1 < KS * KS ? tap + 1 : tap, offn, swn);
#pragma unroll
      for (int c = 0; c < NH; ++c) {
        const int s = tap * NH + c;
        const uint4 bcur = bq[c % D];
#if defined(MZ_LAT_ABLATE) && MZ_LAT_ABLATE == 1
        bq[c % D] = wp[(size_t)((s + D) & 7) * 64];  // ablation: weights from an 8-step (8 KB) hot window
#else
        bq[c % D] = wp[(size_t)(s + D) * 64];
#endif
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, bcur);
        // MFMA on this step's fragment, then issue the next step's read of the same row tile:
        // it has the 4 following MFMAs (~128 cycles) to land.
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
#if defined(MZ_LAT_ABLATE) && MZ_LAT_ABLATE == 3
          asm volatile("" ::"v"(afc[rt]), "v"(bfr));  // ablation: no MFMA
#else
          acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[rt], bfr, acc[rt], 0, 0, 0);
#endif
#if !(defined(MZ_LAT_ABLATE) && MZ_LAT_ABLATE == 2)
          if (c + 1 < NH)
            afn[rt] = *reinterpret_cast<const bf16x8*>(lds + offc[rt] + (((cbase + 2 * (c + 1)) << 4) ^ swc[rt]));
          else
            afn[rt] = *reinterpret_cast<const bf16x8*>(lds + offn[rt] + ((cbase << 4) ^ swn[rt]));
#endif
        }
        // interleave {MFMA, DS read, VALU} x R, then the weight load; the reads' consumers are
        // behind the step barrier, so no MFMA waits on a read issued in its own step
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) afc[rt] = afn[rt];
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) { offc[rt] = offn[rt]; swc[rt] = swn[rt]; }
    }
  }

  // ---- epilogue, staged through LDS: channel-half 0 writes its f32 partial tile, half 1
  // adds its own (each element owned by one lane), then every lane finishes 16-B chunks:
  // + bias (+ act bias) (+ residual, 16-B loads), ReLU, bf16, 16-B stores.
  MZ_STAMP(3);
  uint4 rv[EPT_MAX];
  lat_res_prefetch<NT, MAXROWS>(a, rv, rows, env0, HW, tid);
  __syncthreads();  // every wave is done reading the A tile
  MZ_STAMP(4);
  float* ot = reinterpret_cast<float*>(lds);
  if (active && kh == 0) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) ot[(rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 128 + wq * 32 + l32] = acc[rt][r];
  }
  __syncthreads();
  if (active && kh == 1 && KSPLIT == 2) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float* p = ot + (rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 128 + wq * 32 + l32;
        *p = *p + acc[rt][r];
      }
  }
  __syncthreads();
  lat_epilogue<NT, MAXROWS>(a, ot, rv, rows, env0, HW, tid);
  MZ_STAMP(5);
}

// Variant with 2 column tiles per wave: 4 waves = 2 column halves (64 channels each) x 2
// channel halves of every tap, one wave per SIMD (512-register budget). Each A fragment read
// from LDS feeds 2 MFMAs (half the LDS traffic per FLOP of conv_lat_kernel). Same weight
// packing as the 8-wave kernel (pack_lat ksplit=2).
template <int KS, int CIN>
__global__ __launch_bounds__(256, 1) void conv_lat2_kernel(LatArgs a) {
  constexpr int NC = CIN / 16;
  constexpr int NH = NC / 2;             // k steps per tap per wave
  constexpr int NSW = KS * KS * NH;      // k steps per wave
  constexpr int D = NH >= 8 ? 8 : NH;    // ring depth per column tile
  constexpr int ROWB = CIN * 2;
  constexpr int NCHUNK = CIN / 8;
  constexpr int SMASK = NCHUNK >= 16 ? 15 : NCHUNK - 1;
  constexpr int PAD = KS / 2;
  constexpr int NT = 256;
  static_assert(NH % D == 0, "ring / tap alignment");
  constexpr int LDS_A = (MAXROWS + 1) * ROWB, LDS_C = MAXROWS * 128 * 4;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_A > LDS_C ? LDS_A : LDS_C];
  __shared__ long long envoff[32 * R];
  const int HW = a.H * a.W;
  const int env0 = blockIdx.x * a.E;
  const int nenv = min(a.E, a.B - env0);
  const int rows = nenv * HW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cw = wave & 1, kh = wave >> 1;          // column half (2 tiles), channel half
  const int ct0 = blockIdx.y * 4 + 2 * cw;           // first of this wave's two 32-column tiles
  const bool act0 = ct0 * 32 < a.Cout, act1 = (ct0 + 1) * 32 < a.Cout;
  MZ_STAMP(0);
  const uint4* wp0 = reinterpret_cast<const uint4*>(a.wf) + ((size_t)(act0 ? ct0 : 0) * 2 + kh) * NSW * 64 + lane;
  const uint4* wp1 = reinterpret_cast<const uint4*>(a.wf) + ((size_t)(act1 ? ct0 + 1 : 0) * 2 + kh) * NSW * 64 + lane;
  uint4 bq0[D], bq1[D];
#pragma unroll
  for (int i = 0; i < D; ++i) { bq0[i] = wp0[(size_t)i * 64]; bq1[i] = wp1[(size_t)i * 64]; }
  const float bias0 = a.bias[act0 ? ct0 * 32 + (lane & 31) : 0], bias1 = a.bias[act1 ? ct0 * 32 + 32 + (lane & 31) : 0];

  if (tid < a.E) {
    const int b = env0 + (tid < nenv ? tid : 0);
    long long off = (long long)b * a.in_env_stride;
    if (a.slot) off += (long long)a.slot[b] * a.in_slot_stride;
    envoff[tid] = off;
  }
  __syncthreads();
  constexpr int TOTAL = (MAXROWS + 1) * NCHUNK;
  constexpr int PER = (TOTAL + NT - 1) / NT;
  constexpr int BATCH = PER < 11 ? PER : 11;
#pragma unroll
  for (int base = 0; base < PER; base += BATCH) {
    uint4 v[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int i = (base + u) * NT + tid;
      const int r = i / NCHUNK, c = i % NCHUNK;
      const bool ok = base + u < PER && i < TOTAL && r < rows;
      const int rr = ok ? r : 0;
      const int e = rr / HW, p = rr - (rr / HW) * HW;
      v[u] = *reinterpret_cast<const uint4*>(a.in + envoff[e] + (long long)p * CIN + c * 8);
      if (!ok) v[u] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int i = (base + u) * NT + tid;
      if (base + u < PER && i < TOTAL) {
        const int r = i / NCHUNK, c = i % NCHUNK;
        *reinterpret_cast<uint4*>(lds + r * ROWB + ((c ^ (r & SMASK)) << 4)) = v[u];
      }
    }
  }
  __syncthreads();
  MZ_STAMP(1);

  const int l32 = lane & 31, h = lane >> 5;
  f32x16 acc0[R], acc1[R];
#pragma unroll
  for (int rt = 0; rt < R; ++rt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = rt * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      acc0[rt][i] = (act0 && kh == 0) ? lat_acc_init(a, bias0, row, rows, ct0 * 32 + (lane & 31), env0, HW) : 0.f;
      acc1[rt][i] = (act1 && kh == 0) ? lat_acc_init(a, bias1, row, rows, ct0 * 32 + 32 + (lane & 31), env0, HW) : 0.f;
    }
  {
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
    const int cbase = kh * (2 * NH) + h;
    int offc[R], swc[R], offn[R], swn[R];
    tap_rows(0, offc, swc);
    bf16x8 afc[R], afn[R];
#pragma unroll
    for (int rt = 0; rt < R; ++rt)
      afc[rt] = *reinterpret_cast<const bf16x8*>(lds + offc[rt] + ((cbase << 4) ^ swc[rt]));
    for (int tap = 0; tap < KS * KS; ++tap) {
      tap_rows(tap + 1 < KS * KS ? tap + 1 : tap, offn, swn);
#pragma unroll
      for (int c = 0; c < NH; ++c) {
        const int s = tap * NH + c;
        const bf16x8 b0 = __builtin_bit_cast(bf16x8, bq0[c % D]);
        const bf16x8 b1 = __builtin_bit_cast(bf16x8, bq1[c % D]);
        bq0[c % D] = wp0[(size_t)(s + D) * 64];
        bq1[c % D] = wp1[(size_t)(s + D) * 64];
#pragma unroll
        for (int rt = 0; rt < R; ++rt) {
          acc0[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[rt], b0, acc0[rt], 0, 0, 0);
          acc1[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[rt], b1, acc1[rt], 0, 0, 0);
          if (c + 1 < NH)
            afn[rt] = *reinterpret_cast<const bf16x8*>(lds + offc[rt] + (((cbase + 2 * (c + 1)) << 4) ^ swc[rt]));
          else
            afn[rt] = *reinterpret_cast<const bf16x8*>(lds + offn[rt] + ((cbase << 4) ^ swn[rt]));
        }
#pragma unroll
        for (int rt = 0; rt < R; ++rt) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 0; rt < R; ++rt) afc[rt] = afn[rt];
      }
#pragma unroll
      for (int rt = 0; rt < R; ++rt) { offc[rt] = offn[rt]; swc[rt] = swn[rt]; }
    }
  }

  MZ_STAMP(3);
  uint4 rv[EPT_MAX];
  lat_res_prefetch<NT>(a, rv, rows, env0, HW, tid);
  __syncthreads();
  MZ_STAMP(4);
  float* ot = reinterpret_cast<float*>(lds);
  const int col0 = cw * 64 + l32;
  if (kh == 0) {
#pragma unroll
    for (int rt = 0; rt < R; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        ot[row * 128 + col0] = acc0[rt][r];
        ot[row * 128 + col0 + 32] = acc1[rt][r];
      }
  }
  __syncthreads();
  if (kh == 1) {
#pragma unroll
    for (int rt = 0; rt < R; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        ot[row * 128 + col0] += acc0[rt][r];
        ot[row * 128 + col0 + 32] += acc1[rt][r];
      }
  }
  __syncthreads();
  lat_epilogue<NT>(a, ot, rv, rows, env0, HW, tid);
  MZ_STAMP(5);
}

}  // namespace

// kernel shape, see mzba_conv_lat_set_variant. Per host thread: the learner brackets a minibatch
// with set/restore, and mzba_conv_lat_bn_chunks (which sizes the caller's partial-statistics buffer)
// and the launch that fills it must see the same value even if another host thread (acting beside
// learning) sets its own.
static thread_local int g_lat_variant = 0;

extern "C" {

static int lat_ncu() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

// 0: 8 waves (2 per SIMD: 4 column tiles x 2 channel halves), the default (3-row-tile workgroups
//    where the 5-tile grid would leave CUs idle);
// 1: 4 waves with 2 column tiles each (conv_lat2_kernel, experiment). Same weight packing;
// 2: the default kernel with 5-row-tile workgroups only (A/B reference);
// 3: 3-row-tile workgroups wherever they apply, the two-workgroups-per-CU instance (OCC 2: <= 128 VGPRs, ring depth
//    4, ~56 KiB LDS); the fused BN finaliser (ctr) keeps the one-per-CU instances (its hand-off's condition).
int mzba_conv_lat_set_variant(int v) {
  if (v < 0 || v > 3) return -1;
  g_lat_variant = v;
  return 0;
}
int mzba_conv_lat_get_variant(void) { return g_lat_variant; }

#ifdef MZ_LAT_STAMPS
int mzba_lat_stamps_read(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mz_lat_stamps), sizeof(unsigned long long) * 8 * n);
}
#endif

int mzba_conv_lat_supported(int H, int W, int Cin, int Cout, int ks) {
  const int HW = H * W;
  if (HW > 32 * R || HW <= 0) return 0;
  if (!(Cin == 64 || Cin == 128 || Cin == 256) || Cout % 32 != 0) return 0;
  if (!(ks == 1 || ks == 3)) return 0;
  return 1;
}

// workgroup geometry: envs per workgroup and whether the 3-row-tile kernel runs
static void lat_geometry(int B, int H, int W, int Cin, int Cout, int& E, bool& rt3) {
  const int HW = H * W;
  const int ny = (Cout + 127) / 128;
  E = (32 * R) / HW;
  // 3-tile workgroups (E3 envs) when the 5-tile grid leaves CUs idle and the smaller tiles add
  // workgroups (learner B = 512 at 4x5: 128 -> 256); the per-element arithmetic is the same
  const int E3 = (32 * 3) / HW;
  rt3 = g_lat_variant == 0 && E3 >= 1 && (long long)((B + E - 1) / E) * ny < lat_ncu() &&
        (B + E3 - 1) / E3 > (B + E - 1) / E && Cin >= 128;
  if (g_lat_variant == 3 && E3 >= 1 && Cin >= 128) rt3 = true;
  if (rt3) E = E3;
}

static int lat_launch(LatArgs& a, hipStream_t stream) {
  bool rt3;
  lat_geometry(a.B, a.H, a.W, a.Cin, a.Cout, a.E, rt3);
  const int ks = a.ks, Cin = a.Cin;
  dim3 grid((a.B + a.E - 1) / a.E, (a.Cout + 127) / 128);
  const int v = g_lat_variant;
#define MZ_LAT(KS_, CIN_, W_, D_) \
  if (ks == KS_ && Cin == CIN_) { hipLaunchKernelGGL((conv_lat_kernel<KS_, CIN_, W_, D_>), grid, dim3(64 * W_), 0, stream, a); }
#define MZ_LAT3(KS_, CIN_)                                                                                      \
  if (ks == KS_ && Cin == CIN_) {                                                                               \
    if (v == 3 && !a.ctr)                                                                                       \
      hipLaunchKernelGGL((conv_lat_kernel<KS_, CIN_, 8, 4, 3, 2>), grid, dim3(512), 0, stream, a);              \
    else                                                                                                        \
      hipLaunchKernelGGL((conv_lat_kernel<KS_, CIN_, 8, 8, 3>), grid, dim3(512), 0, stream, a);                 \
  }
  if (v == 1) {
    if (a.smode) return -4;  // the fused statistics ride on the 8-wave kernel only
    if (ks == 3 && Cin == 256) hipLaunchKernelGGL((conv_lat2_kernel<3, 256>), grid, dim3(256), 0, stream, a);
    else if (ks == 1 && Cin == 256) hipLaunchKernelGGL((conv_lat2_kernel<1, 256>), grid, dim3(256), 0, stream, a);
    else return -4;
  } else if (rt3) {
    MZ_LAT3(3, 256) else MZ_LAT3(1, 256) else MZ_LAT3(3, 128) else MZ_LAT3(1, 128)
  } else {
    MZ_LAT(3, 256, 8, 8) else MZ_LAT(1, 256, 8, 8) else MZ_LAT(3, 128, 8, 8) else MZ_LAT(1, 128, 8, 8)
    else MZ_LAT(3, 64, 8, 8) else MZ_LAT(1, 64, 8, 8)
  }
#undef MZ_LAT
#undef MZ_LAT3
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_conv_lat(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                  const void* wf, const float* bias, const float* act_bias, const int32_t* act, int A,
                  const void* res, void* out, int B, int H, int W, int Cin, int Cout, int ks, int relu,
                  hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && mzba_conv_lat_supported(H, W, Cin, Cout, ks), -1);
  MZ_CHECK_ARG(!act_bias || (act && A > 0), -3);
  LatArgs a{(const bf16_t*)in, in_env_stride, slot, in_slot_stride, (const bf16_t*)wf, bias, act_bias, act, A,
            (const bf16_t*)res, (bf16_t*)out, B, H, W, Cin, Cout, ks, relu, 0};
  return lat_launch(a, stream);
}

int mzba_conv_lat_bn_chunks(int B, int H, int W, int Cin, int Cout, int ks, int* nchunk, int* rpc) {
  MZ_CHECK_ARG(B > 0 && nchunk && rpc && mzba_conv_lat_supported(H, W, Cin, Cout, ks), -1);
  int E;
  bool rt3;
  lat_geometry(B, H, W, Cin, Cout, E, rt3);
  *nchunk = (B + E - 1) / E;
  *rpc = E * H * W;
  return 0;
}

int mzba_conv_lat_bn(const void* in, const void* wf, const float* bias, const void* res, void* out, int B, int H,
                     int W, int Cin, int Cout, int ks, int mode, float* part, const void* y, const void* x,
                     const float* mean, const float* pstats, const void* pres, int prelu, void* pout,
                     const float* pcoef, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && in && wf && bias && out && mzba_conv_lat_supported(H, W, Cin, Cout, ks), -1);
  MZ_CHECK_ARG(Cout % 128 == 0 && (mode == 0 || (part && (mode == 1 || (mode == 2 && y && x && mean)))), -3);
  MZ_CHECK_ARG(!pstats || pout, -3);
  MZ_CHECK_ARG(!pcoef || (pstats && pres), -3);
  LatArgs a{(const bf16_t*)in, (long long)H * W * Cin, nullptr, 0, (const bf16_t*)wf, bias, nullptr, nullptr, 0,
            (const bf16_t*)res, (bf16_t*)out, B, H, W, Cin, Cout, ks, 0, 0,
            mode, (float2*)part, (const bf16_t*)y, (const bf16_t*)x, mean,
            pstats, (const bf16_t*)pres, prelu, (bf16_t*)pout, pcoef};
  return lat_launch(a, stream);
}

// mzba_conv_lat_bn plus the consuming BatchNorm's finaliser in the same launch (lat_bn_finish): mode 1 writes that
// BN's stats [4][Cout] and updates its running statistics (run_mean / run_var optional) as mzba_bn_stats_final does;
// mode 2 reads its stats and adds to dgamma / dbeta and writes coef [3][Cout] as mzba_bn_backward_coef does. ctr:
// Cout / 128 unsigned words, zero at entry and zero again at exit (the launch's last workgroups reset them), never
// shared by two launches in flight. The 8-wave kernels only (variant 0 / 2).
int mzba_conv_lat_bn_fin(const void* in, const void* wf, const float* bias, const void* res, void* out, int B, int H,
                         int W, int Cin, int Cout, int ks, int mode, float* part, const void* y, const void* x,
                         const float* mean, const float* pstats, const void* pres, int prelu, void* pout,
                         const float* pcoef, unsigned* ctr, float eps, float momentum, const float* gamma,
                         const float* beta, float* fstats, float* run_mean, float* run_var, float* dgamma, float* dbeta,
                         float* coef, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && in && wf && bias && out && mzba_conv_lat_supported(H, W, Cin, Cout, ks), -1);
  MZ_CHECK_ARG(Cout % 128 == 0 && part && (mode == 1 || (mode == 2 && y && x && mean)), -3);
  MZ_CHECK_ARG(!pstats || pout, -3);
  MZ_CHECK_ARG(!pcoef || (pstats && pres), -3);
  MZ_CHECK_ARG(ctr && fstats && g_lat_variant != 1, -3);
  MZ_CHECK_ARG(mode == 1 ? (gamma && beta && (!run_mean || run_var)) : (dgamma && dbeta && coef), -3);
  LatArgs a{(const bf16_t*)in, (long long)H * W * Cin, nullptr, 0, (const bf16_t*)wf, bias, nullptr, nullptr, 0,
            (const bf16_t*)res, (bf16_t*)out, B, H, W, Cin, Cout, ks, 0, 0,
            mode, (float2*)part, (const bf16_t*)y, (const bf16_t*)x, mean,
            pstats, (const bf16_t*)pres, prelu, (bf16_t*)pout, pcoef,
            ctr, eps, momentum, gamma, beta, fstats, run_mean, run_var, dgamma, dbeta, coef};
  return lat_launch(a, stream);
}

}  // extern "C"
