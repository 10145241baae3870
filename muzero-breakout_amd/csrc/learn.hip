// Learner kernels: one minibatch of RLSystem._training_stage
// (train_torch.py:380-407) = _k_step_rollout forward with train-mode BatchNorm, loss_fn, the
// backward pass and the Adam step, on NHWC activations (T = f32 for parity, bf16 for
// throughput; statistics, gradients and parameters are f32 throughout).
//
// The convolutions themselves run on conv_igemm_kernel (conv.hip): forward with the f32 master
// weights (or their bf16 cast), input gradients as a convolution of the output gradient with
// the flipped, transposed weights (conv_wt_kernel packs them every step). This file holds what
// is specific to training:
//   bn_stats_*        batch mean / biased variance per channel (chunk-wise mean + M2, combined
//                     with Chan's formula in double), running-stat update (networks.py BN layers
//                     in train mode, momentum 0.1, unbiased running variance);
//   bn_apply          y = x * (gamma * invstd) + (beta - mean * gamma * invstd) (+ residual) (ReLU);
//   bn_bwd_*          g = dy * [y > 0] (in place), dgamma / dbeta, dx = (g - (x - mean) k - mean_g)
//                     * gamma * invstd with k = sum(g (x - mean)) invstd^2 / N (torch's CPU order);
//   conv_wgrad        dW[co][tap][ci] = sum_m dY[m][co] X_tap[m][ci] (+ conv bias grad), split
//                     over m into deterministic partials, then reduced into the gradient buffer;
//   scale_fwd / bwd   MuZeroAgent._scale_state (networks.py:314-328) with the first min / max
//                     index in NCHW flatten order (torch.min/max(dim) semantics) for the backward;
//   linear_*          the heads' nn.Linear on an NHWC image (weights kept in [o][pixel][channel]);
//   loss              supports_representation (utils.py:30-64) + log_softmax + KL(batchmean)
//                     for reward / value / policy and their logit gradients (loss_fn :33-66);
//   adam              torch.optim.Adam(lr, weight_decay = 1e-4) single-tensor update (networks.py:268).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

template <typename T> MZ_DEV float ld(const T* p) { return ElemIO<T>::load(p); }
template <typename T> MZ_DEV void st(T* p, float v) { ElemIO<T>::store(p, v); }

// ------------------------------------------------------------------ BatchNorm statistics
// 4 consecutive channels per thread (C % 4 == 0): f32 float4 / bf16 8-byte loads.
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  static MZ_DEV float4 load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static MZ_DEV void store(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
};
template <> struct Vec4<bf16_t> {
  static MZ_DEV float4 load(const bf16_t* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
  }
  static MZ_DEV void store(bf16_t* p, float4 v) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  }
};
MZ_DEV float4 f4add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// part[chunk][c] = (chunk mean, chunk M2) over rows [chunk*rpc, min(M, (chunk+1)*rpc)).
// 256 threads = (channel quads of a 64-channel group = 16) x 16 row lanes.
constexpr int BN_RPC = 64;
constexpr int BN_FK = 8;  // chunks per lane the BN finalisers load ahead (nchunk <= 512 in one round trip)
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const T* __restrict__ x, int M, int C, int rpc,
                                                               float2* __restrict__ part) {
  __shared__ float4 red[16][16];
  const int tq = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + tq * 4;
  const int r0 = blockIdx.y * rpc, r1 = min(M, r0 + rpc);
  const int n = r1 - r0;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < C)
    for (int r = r0 + ty; r < r1; r += 16) s = f4add(s, Vec4<T>::load(x + (size_t)r * C + c));
  red[ty][tq] = s;
  __syncthreads();
  float4 t = red[0][tq];
  for (int k = 1; k < 16; ++k) t = f4add(t, red[k][tq]);
  const float4 mean = make_float4(t.x / n, t.y / n, t.z / n, t.w / n);
  __syncthreads();
  float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < C)
    for (int r = r0 + ty; r < r1; r += 16) {
      const float4 v = Vec4<T>::load(x + (size_t)r * C + c);
      const float4 d = make_float4(v.x - mean.x, v.y - mean.y, v.z - mean.z, v.w - mean.w);
      q = make_float4(q.x + d.x * d.x, q.y + d.y * d.y, q.z + d.z * d.z, q.w + d.w * d.w);
    }
  red[ty][tq] = q;
  __syncthreads();
  if (ty == 0 && c < C) {
    float4 m2 = red[0][tq];
    for (int k = 1; k < 16; ++k) m2 = f4add(m2, red[k][tq]);
    float2* o = part + (size_t)blockIdx.y * C + c;
    o[0] = make_float2(mean.x, m2.x);
    o[1] = make_float2(mean.y, m2.y);
    o[2] = make_float2(mean.z, m2.z);
    o[3] = make_float2(mean.w, m2.w);
  }
}

// combine the chunks (Chan et al., in double) -> mean, invstd, alpha = gamma*invstd,
// beta' = beta - mean*alpha; running stats: r = momentum*stat + (1 - momentum)*r (unbiased var).
// One wave per channel: lane l folds chunks l, l+64, ...; then a fixed butterfly over the lanes.
MZ_DEV void chan_combine(double& n, double& mean, double& m2, double nb, double mb, double m2b) {
  if (nb == 0) return;
  const double tot = n + nb, d = mb - mean;
  mean += d * nb / tot;
  m2 += m2b + d * d * n * nb / tot;
  n = tot;
}

__global__ __launch_bounds__(64) void bn_stats_final_kernel(const float2* __restrict__ part, int nchunk, int rpc, int M,
                                                            int C, float eps, float momentum,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float* __restrict__ stats,
                                                            float* __restrict__ run_mean, float* __restrict__ run_var) {
  const int c = blockIdx.x, lane = threadIdx.x;
  // the per-channel operands of the tail, loaded with the partials (after the butterfly each was one more
  // memory round trip on the chain)
  const float g_c = gamma[c], b_c = beta[c];
  const float rm_c = run_mean ? run_mean[c] : 0.f, rv_c = run_mean ? run_var[c] : 0.f;
  double n = 0, mean = 0, m2 = 0;
  // the lane's chunks l, l + 64, ... (up to BN_FK of them) are all loaded before the first fold: a rolled
  // load-then-fold loop waited one memory round trip per chunk. The folds keep their order (the same sums)
  float2 pv[BN_FK];
#pragma unroll
  for (int i = 0; i < BN_FK; ++i) pv[i] = lane + 64 * i < nchunk ? part[(size_t)(lane + 64 * i) * C + c] : float2{};
#pragma unroll
  for (int i = 0; i < BN_FK; ++i) {
    const int k = lane + 64 * i;
    if (k < nchunk) chan_combine(n, mean, m2, (double)min(rpc, M - k * rpc), (double)pv[i].x, (double)pv[i].y);
  }
  for (int k = lane + 64 * BN_FK; k < nchunk; k += 64) {
    const float2 p = part[(size_t)k * C + c];
    chan_combine(n, mean, m2, (double)min(rpc, M - k * rpc), (double)p.x, (double)p.y);
  }
  for (int o = 1; o < 64; o <<= 1) {
    const double n2 = __shfl_xor(n, o), mean2 = __shfl_xor(mean, o), m22 = __shfl_xor(m2, o);
    chan_combine(n, mean, m2, n2, mean2, m22);
  }
  if (lane) return;
  const float var = (float)(m2 / M);
  const float invstd = (float)(1.0 / sqrt((double)var + (double)eps));
  const float alpha = invstd * g_c;
  const float fm = (float)mean;
  stats[c] = fm;                 // mean
  stats[C + c] = invstd;         // invstd
  stats[2 * C + c] = alpha;      // gamma * invstd
  stats[3 * C + c] = b_c - fm * alpha;
  if (run_mean) {
    run_mean[c] = (float)((double)momentum * mean + (1.0 - (double)momentum) * (double)rm_c);
    const double unbiased = M > 1 ? m2 / (double)(M - 1) : m2;
    run_var[c] = (float)((double)momentum * unbiased + (1.0 - (double)momentum) * (double)rv_c);
  }
}

// y = x*alpha + beta' (+ res) (ReLU); 4 channels per thread (C % 4 == 0)
template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ x, const float* __restrict__ stats,
                                                       const T* res, int relu, T* out, int M, int C) {
  const size_t n4 = (size_t)M * C / 4;
  const float* alpha = stats + 2 * C;
  const float* beta = stats + 3 * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const size_t e = i * 4;
    const int c = (int)(e % C);
    const float4 v = Vec4<T>::load(x + e);
    const float4 a = *reinterpret_cast<const float4*>(alpha + c), b = *reinterpret_cast<const float4*>(beta + c);
    float4 y = make_float4(v.x * a.x + b.x, v.y * a.y + b.y, v.z * a.z + b.z, v.w * a.w + b.w);
    if (res) y = f4add(y, Vec4<T>::load(res + e));
    if (relu) y = make_float4(fmaxf(y.x, 0.f), fmaxf(y.y, 0.f), fmaxf(y.z, 0.f), fmaxf(y.w, 0.f));
    Vec4<T>::store(out + e, y);
  }
}

// ------------------------------------------------------------------ BatchNorm backward
// g = dy * [y > 0] (written back to dy when y != null); part[chunk][c] = (sum g, sum g (x - mean))
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(T* __restrict__ dy, const T* __restrict__ y,
                                                             const T* __restrict__ x, const float* __restrict__ stats,
                                                             int M, int C, int rpc, float2* __restrict__ part) {
  __shared__ float4 red[2][16][16];
  const int tq = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + tq * 4;
  const int r0 = blockIdx.y * rpc, r1 = min(M, r0 + rpc);
  float4 sg = make_float4(0.f, 0.f, 0.f, 0.f), sd = sg;
  if (c < C) {
    const float4 mean = *reinterpret_cast<const float4*>(stats + c);
    for (int r = r0 + ty; r < r1; r += 16) {
      const size_t i = (size_t)r * C + c;
      float4 g = Vec4<T>::load(dy + i);
      if (y) {
        const float4 yv = Vec4<T>::load(y + i);
        if (!(yv.x > 0.f)) g.x = 0.f;
        if (!(yv.y > 0.f)) g.y = 0.f;
        if (!(yv.z > 0.f)) g.z = 0.f;
        if (!(yv.w > 0.f)) g.w = 0.f;
        Vec4<T>::store(dy + i, g);
      }
      const float4 xv = Vec4<T>::load(x + i);
      sg = f4add(sg, g);
      sd = make_float4(sd.x + g.x * (xv.x - mean.x), sd.y + g.y * (xv.y - mean.y), sd.z + g.z * (xv.z - mean.z),
                       sd.w + g.w * (xv.w - mean.w));
    }
  }
  red[0][ty][tq] = sg;
  red[1][ty][tq] = sd;
  __syncthreads();
  if (ty == 0 && c < C) {
    float4 a = red[0][0][tq], b = red[1][0][tq];
    for (int k = 1; k < 16; ++k) { a = f4add(a, red[0][k][tq]); b = f4add(b, red[1][k][tq]); }
    float2* o = part + (size_t)blockIdx.y * C + c;
    o[0] = make_float2(a.x, b.x);
    o[1] = make_float2(a.y, b.y);
    o[2] = make_float2(a.z, b.z);
    o[3] = make_float2(a.w, b.w);
  }
}

// dgamma += dot*invstd, dbeta += sum g; coef = (mean_g, k = dot*invstd^2/N, gamma*invstd).
// One wave per channel, double sums, fixed butterfly order.
__global__ __launch_bounds__(64) void bn_bwd_final_kernel(const float2* __restrict__ part, int nchunk, int M, int C,
                                                          const float* __restrict__ stats, float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta, float* __restrict__ coef) {
  const int c = blockIdx.x, lane = threadIdx.x;
  // the tail's per-channel operands, loaded with the partials (as bn_stats_final_kernel)
  const float invstd = stats[C + c], alpha = stats[2 * C + c], dg_c = dgamma[c], db_c = dbeta[c];
  double sg = 0, dot = 0;
  float2 pv[BN_FK];  // loaded before the first add, as bn_stats_final_kernel (the same sums)
#pragma unroll
  for (int i = 0; i < BN_FK; ++i) pv[i] = lane + 64 * i < nchunk ? part[(size_t)(lane + 64 * i) * C + c] : float2{};
#pragma unroll
  for (int i = 0; i < BN_FK; ++i)
    if (lane + 64 * i < nchunk) {
      sg += pv[i].x;
      dot += pv[i].y;
    }
  for (int k = lane + 64 * BN_FK; k < nchunk; k += 64) {
    const float2 p = part[(size_t)k * C + c];
    sg += p.x;
    dot += p.y;
  }
  for (int o = 1; o < 64; o <<= 1) {
    sg += __shfl_xor(sg, o);
    dot += __shfl_xor(dot, o);
  }
  if (lane) return;
  dgamma[c] = dg_c + (float)dot * invstd;
  dbeta[c] = db_c + (float)sg;
  coef[c] = (float)(sg / M);
  coef[C + c] = (float)dot * invstd * invstd / (float)M;
  coef[2 * C + c] = alpha;
}

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ g, const T* __restrict__ x,
                                                           const float* __restrict__ stats,
                                                           const float* __restrict__ coef, T* __restrict__ dx, int M,
                                                           int C) {
  const size_t n4 = (size_t)M * C / 4;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const size_t e = i * 4;
    const int c = (int)(e % C);
    const float4 gv = Vec4<T>::load(g + e), xv = Vec4<T>::load(x + e);
    const float4 mu = *reinterpret_cast<const float4*>(stats + c);
    const float4 mg = *reinterpret_cast<const float4*>(coef + c);
    const float4 k = *reinterpret_cast<const float4*>(coef + C + c);
    const float4 s = *reinterpret_cast<const float4*>(coef + 2 * C + c);
    Vec4<T>::store(dx + e, make_float4(((gv.x - (xv.x - mu.x) * k.x) - mg.x) * s.x, ((gv.y - (xv.y - mu.y) * k.y) - mg.y) * s.y,
                                       ((gv.z - (xv.z - mu.z) * k.z) - mg.z) * s.z, ((gv.w - (xv.w - mu.w) * k.w) - mg.w) * s.w));
  }
}

// ------------------------------------------------------------------ conv weight packs
// wt[ci][tap][co] = w[co][taps-1-tap][ci] for ci < cin_used (input-gradient conv), or a plain
// cast wt = w (mode 0). w: f32 master [Cout][taps][Cin].
template <typename T>
__global__ void conv_wt_kernel(const float* __restrict__ w, T* __restrict__ wt, int Cout, int taps, int Cin,
                               int cin_used, int flip) {
  const size_t n = flip ? (size_t)cin_used * taps * Cout : (size_t)Cout * taps * Cin;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (!flip) {
      st(wt + i, w[i]);
    } else {
      const int co = (int)(i % Cout);
      const size_t q = i / Cout;
      const int tap = (int)(q % taps), ci = (int)(q / taps);
      st(wt + i, w[((size_t)co * taps + (taps - 1 - tap)) * Cin + ci]);
    }
  }
}

// bf16 weight packs for the latent / band conv kernels, straight from the f32 master weights:
// logical W'[n][tap][c] = flip ? w[c][taps-1-tap][n] : w[n][tap][c] (n < N rows, c < Cc).
// layout 1 (conv_lat, agent.pack_lat): out[ct][kh][tap][cc][h][r][j] = W'[32ct + r][tap][kh Cc/2 + 16cc + 8h + j];
// layout 2 (tower / band, agent.pack_tower_conv, 3x3): out[ct][s][g][r][j] = W'[16ct + r] at
// k' = 32s + 8g + j with taps in (dx, dy) order: q = k' / Cc, tap = (q % 3) * 3 + q / 3.
// `pad` zero elements follow (the kernels' weight-ring overrun).
__global__ void conv_pack_kernel(const float* __restrict__ w, bf16_t* __restrict__ out, int Cout, int taps, int Cin,
                                 int N, int Cc, int flip, int layout, size_t pad) {
  const size_t n_el = (size_t)N * taps * Cc;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_el + pad; i += (size_t)gridDim.x * blockDim.x) {
    if (i >= n_el) { out[i] = 0; continue; }
    int n, tap, c;
    size_t q = i;
    if (layout == 1) {
      const int j = (int)(q % 8); q /= 8;
      const int r = (int)(q % 32); q /= 32;
      const int h = (int)(q % 2); q /= 2;
      const int cc = (int)(q % (Cc / 32)); q /= (Cc / 32);
      tap = (int)(q % taps); q /= taps;
      const int kh = (int)(q % 2);
      const int ct = (int)(q / 2);
      n = 32 * ct + r;
      c = kh * (Cc / 2) + 16 * cc + 8 * h + j;
    } else {
      const int j = (int)(q % 8); q /= 8;
      const int r = (int)(q % 16); q /= 16;
      const int g = (int)(q % 4); q /= 4;
      const size_t nk = (size_t)taps * Cc / 32;
      const int s_ = (int)(q % nk);
      const int ct = (int)(q / nk);
      n = 16 * ct + r;
      const int k = 32 * s_ + 8 * g + j;
      const int qq = k / Cc;
      c = k - qq * Cc;
      tap = (qq % 3) * 3 + qq / 3;
    }
    const float v = flip ? w[((size_t)c * taps + (taps - 1 - tap)) * Cin + n] : w[((size_t)n * taps + tap) * Cin + c];
    out[i] = f32_to_bf16(v);
  }
}

// Many packs in one launch (the learner's per-minibatch packs of every conv: one launch per PK_MAX of them instead of
// one each): blockIdx.y = job, a thread per 8 consecutive output elements (8 consecutive c of one (n, tap): Cc % 32
// == 0 and pad % 8 == 0), the same element values as conv_pack_kernel, one 16-B store.
struct PackJob {
  const float* w;
  bf16_t* out;
  int Cout, taps, Cin, N, Cc, flip, layout, pad;
};
constexpr int PK_MAX = 32;
struct PackJobs {
  PackJob j[PK_MAX];
};
__global__ __launch_bounds__(256) void conv_pack_multi_kernel(PackJobs js) {
  const PackJob& jb = js.j[blockIdx.y];
  const int taps = jb.taps, Cc = jb.Cc, Cin = jb.Cin;
  const int n_el = jb.N * taps * Cc, ng = (n_el + jb.pad) / 8;
  for (int g8 = blockIdx.x * blockDim.x + threadIdx.x; g8 < ng; g8 += gridDim.x * blockDim.x) {
    const int i = 8 * g8;
    uint4 o = make_uint4(0, 0, 0, 0);
    if (i < n_el) {
      int n, tap, c, q = i / 8;
      if (jb.layout == 1) {
        const int r = q % 32; q /= 32;
        const int h = q % 2; q /= 2;
        const int cc = q % (Cc / 32); q /= Cc / 32;
        tap = q % taps; q /= taps;
        const int kh = q % 2, ct = q / 2;
        n = 32 * ct + r;
        c = kh * (Cc / 2) + 16 * cc + 8 * h;
      } else {
        const int r = q % 16; q /= 16;
        const int g = q % 4; q /= 4;
        const int nk = taps * Cc / 32, s_ = q % nk, ct = q / nk;
        n = 16 * ct + r;
        const int k = 32 * s_ + 8 * g, qq = k / Cc;
        c = k - qq * Cc;
        tap = (qq % 3) * 3 + qq / 3;
      }
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = jb.flip ? jb.w[((size_t)(c + j) * taps + (taps - 1 - tap)) * Cin + n] : jb.w[((size_t)n * taps + tap) * Cin + c + j];
      o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
    *reinterpret_cast<uint4*>(jb.out + i) = o;
  }
}

// ------------------------------------------------------------------ conv weight gradient
// One workgroup: a 64 (co) x 64 (ci) tile of one tap over a chunk of m rows, 4 waves as 2x2 of
// 32x32 (2x2 MFMA 16x16 tiles). K = m in steps of 16 rows staged through LDS.
// f32: v_mfma_f32_16x16x4_f32 (lane: row l&15, k = l>>4). bf16: rows are widened to f32 in LDS.
constexpr int WG_ROWS = 16, WG_LD = 80;  // LDS row stride (floats): 16-bank shift per k row

template <typename T>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy, int B,
                                                         int H, int W, int Cin, int Cout, int ks, int rows_per_split,
                                                         float* __restrict__ part, float* __restrict__ bpart) {
  __shared__ float la[2][WG_ROWS][WG_LD];  // dY tile [m][co]
  __shared__ float lb[2][WG_ROWS][WG_LD];  // X tile  [m][ci]
  const int taps = ks * ks, pad = ks / 2;
  const int nci = (Cin + 63) / 64;
  int t = blockIdx.x;
  const int cit = t % nci; t /= nci;
  const int tap = t % taps; t /= taps;
  const int cot = t;
  const int split = blockIdx.y;
  const int HW = H * W, M = B * HW;
  const int m0 = split * rows_per_split, m1 = min(M, m0 + rows_per_split);
  const int ky = tap / ks - pad, kx = tap % ks - pad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  // staging: thread -> (row lr = tid >> 4, 4 channels at 4*(tid & 15))
  const int lr = tid >> 4, lc = (tid & 15) * 4;
  const int co_s = cot * 64 + lc, ci_s = cit * 64 + lc;
  float4 va, vb;
  auto load = [&](int mb) {
    const int m = mb + lr;
    va = make_float4(0.f, 0.f, 0.f, 0.f);
    vb = va;
    if (m < m1) {
      const int b = m / HW, p = m - b * HW, yy = p / W, xx = p - yy * W;
      const T* d = dy + (size_t)m * Cout + co_s;
      if (co_s < Cout) va = make_float4(ld(d), ld(d + 1), ld(d + 2), ld(d + 3));
      const int sy = yy + ky, sx = xx + kx;
      if (ci_s < Cin && sy >= 0 && sy < H && sx >= 0 && sx < W) {
        const T* s = x + ((size_t)b * HW + sy * W + sx) * Cin + ci_s;
        vb = make_float4(ld(s), ld(s + 1), ld(s + 2), ld(s + 3));
      }
    }
  };
  auto store = [&](int buf) {
    *reinterpret_cast<float4*>(&la[buf][lr][lc]) = va;
    *reinterpret_cast<float4*>(&lb[buf][lr][lc]) = vb;
  };
  const bool do_bias = bpart && tap == 0 && cit == 0;
  typedef __attribute__((ext_vector_type(4))) float f4;
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = (m1 - m0 + WG_ROWS - 1) / WG_ROWS;
  if (nsteps > 0) {
    load(m0);
    store(0);
  }
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  float4 bacc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (do_bias) { bacc.x += va.x; bacc.y += va.y; bacc.z += va.z; bacc.w += va.w; }
    if (s + 1 < nsteps) load(m0 + (s + 1) * WG_ROWS);
#pragma unroll
    for (int kk = 0; kk < WG_ROWS / 4; ++kk) {
      const int r = kk * 4 + fk;
      float a[2], bb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = la[buf][r][wr * 32 + i * 16 + fr];
#pragma unroll
      for (int j = 0; j < 2; ++j) bb[j] = lb[buf][r][wc * 32 + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }
  // D[row = co 4*fk + r][col = ci fr] of each 16x16 tile
  const size_t K = (size_t)taps * Cin;
  float* outp = part + (size_t)split * Cout * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ci = cit * 64 + wc * 32 + j * 16 + fr;
      if (ci >= Cin) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cot * 64 + wr * 32 + i * 16 + 4 * fk + r;
        if (co < Cout) outp[(size_t)co * K + (size_t)tap * Cin + ci] = acc[i][j][r];
      }
    }
  if (do_bias) {  // reduce the 16 row lanes of each channel group through LDS
    __shared__ float4 bred[16][16];
    bred[lr][tid & 15] = bacc;
    __syncthreads();
    if (tid < 16) {
      float4 s = bred[0][tid];
      for (int r = 1; r < 16; ++r) { s.x += bred[r][tid].x; s.y += bred[r][tid].y; s.z += bred[r][tid].z; s.w += bred[r][tid].w; }
      const int co = cot * 64 + tid * 4;
      float* bp = bpart + (size_t)split * Cout;
      if (co < Cout) { bp[co] = s.x; bp[co + 1] = s.y; bp[co + 2] = s.z; bp[co + 3] = s.w; }
    }
  }
}

// bf16: v_mfma_f32_16x16x32_bf16 with both operands read by ds_read_b64_tr_b16 from row-major
// [m][channel] LDS tiles (rows staged straight from HBM, 16-B chunks). A = dY^T (co x m), B = X_tap
// (m x ci). Lane group g (lanes 16g..16g+15) takes k rows {4g..4g+3} and {16+4g..16+4g+3} of each
// 32-row k step (the same permutation for A and B); a 160-B row stride makes each 32-lane half's
// eight rows hit disjoint banks.
constexpr int WB_M = 64, WB_LD = 80;  // rows per stage, bf16 per LDS row
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

MZ_DEV bf16x8_t tr_frag(const bf16_t* base) {  // base: this lane's address for the first 4 rows
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + 16 * WB_LD));
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, r);  // bit pattern, not a numeric short -> bf16 conversion
}

__global__ __launch_bounds__(256) void conv_wgrad_bf16_kernel(const bf16_t* __restrict__ x,
                                                              const bf16_t* __restrict__ dy, int B, int H, int W,
                                                              int Cin, int Cout, int ks, int rows_per_split,
                                                              float* __restrict__ part, float* __restrict__ bpart) {
  __shared__ __attribute__((aligned(16))) bf16_t la[2][WB_M][WB_LD];
  __shared__ __attribute__((aligned(16))) bf16_t lb[2][WB_M][WB_LD];
  __shared__ float bred[32][64];
  const int taps = ks * ks, pad = ks / 2;
  const int nci = (Cin + 63) / 64;
  int t = blockIdx.x;
  const int cit = t % nci; t /= nci;
  const int tap = t % taps; t /= taps;
  const int cot = t;
  const int split = blockIdx.y;
  const int HW = H * W, M = B * HW;
  const int m0 = split * rows_per_split, m1 = min(M, m0 + rows_per_split);
  const int ky = tap / ks - pad, kx = tap % ks - pad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  // staging: chunk c = tid + 256u (u = 0, 1): row c >> 3, 8 channels at 8*(c & 7)
  const int ch = tid & 7;
  const int co_s = cot * 64 + ch * 8, ci_s = cit * 64 + ch * 8;
  uint4 va[2], vb[2];
  auto load = [&](int mb) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = mb + ((tid + 256 * u) >> 3);
      va[u] = make_uint4(0, 0, 0, 0);
      vb[u] = va[u];
      if (m < m1) {
        const int b = m / HW, p = m - b * HW, yy = p / W, xx = p - yy * W;
        if (co_s < Cout) va[u] = *reinterpret_cast<const uint4*>(dy + (size_t)m * Cout + co_s);
        const int sy = yy + ky, sx = xx + kx;
        if (ci_s < Cin && sy >= 0 && sy < H && sx >= 0 && sx < W)
          vb[u] = *reinterpret_cast<const uint4*>(x + ((size_t)b * HW + sy * W + sx) * Cin + ci_s);
      }
    }
  };
  const bool do_bias = bpart && tap == 0 && cit == 0;
  float bacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bacc[j] = 0.f;
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = (tid + 256 * u) >> 3;
      *reinterpret_cast<uint4*>(&la[buf][r][ch * 8]) = va[u];
      *reinterpret_cast<uint4*>(&lb[buf][r][ch * 8]) = vb[u];
      if (do_bias) {
        const bf16_t* e = reinterpret_cast<const bf16_t*>(&va[u]);
#pragma unroll
        for (int j = 0; j < 8; ++j) bacc[j] += bf16_to_f32(e[j]);
      }
    }
  };
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int nsteps = (m1 - m0 + WB_M - 1) / WB_M;
  if (nsteps > 0) {
    load(m0);
    store(0);
  }
  __syncthreads();
  // transposed-read lane address: group g = lane >> 4 takes rows 4g + q, q = (lane & 15) >> 2,
  // columns 4p.. (p = lane & 3) of its 16-column block
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) load(m0 + (s + 1) * WB_M);
#pragma unroll
    for (int kk = 0; kk < WB_M / 32; ++kk) {
      const int row = kk * 32 + 4 * g + q;
      bf16x8_t a[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = tr_frag(&la[buf][row][wr * 32 + i * 16 + 4 * pp]);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = tr_frag(&lb[buf][row][wc * 32 + j * 16 + 4 * pp]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }
  const size_t K = (size_t)taps * Cin;
  float* outp = part + (size_t)split * Cout * K;
  const int fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ci = cit * 64 + wc * 32 + j * 16 + fr;
      if (ci >= Cin) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cot * 64 + wr * 32 + i * 16 + 4 * fk + r;
        if (co < Cout) outp[(size_t)co * K + (size_t)tap * Cin + ci] = acc[i][j][r];
      }
    }
  if (do_bias) {  // 32 row lanes per channel group -> column sums
#pragma unroll
    for (int j = 0; j < 8; ++j) bred[tid >> 3][ch * 8 + j] = bacc[j];
    __syncthreads();
    if (tid < 64) {
      float sum = 0.f;
      for (int r = 0; r < 32; ++r) sum += bred[r][tid];
      const int co = cot * 64 + tid;
      if (co < Cout) bpart[(size_t)split * Cout + co] = sum;
    }
  }
}

// bf16 3x3 weight gradient over whole images: one workgroup = a 64 (co) x 64 (ci) tile for ALL 9
// taps, over E envs per LDS stage. Each env's image is staged once with a zero border (Hp = H + 2,
// Wp = W + 2 rows of 64 channels); the contraction index k runs over the H x Wp interior-row
// positions (border columns carry dY = 0), so tap (dy, dx) is the constant row offset
// dy * Wp + dx into the bordered X image: every 4-row transposed-read block stays contiguous and
// dY / X are read from HBM once per tile instead of once per tap.
constexpr int WI_LD = 80;        // bf16 per LDS row (160 B, the transposed-read bank layout above)
constexpr int WI_LEAD = 8;       // zero rows before the X images (tap offsets reach -Wp - 1)
constexpr int WI_PF = 24;        // staging chunks per 256 threads (KS + XR <= 768 rows)

// up to WG_MAXSEG (x, dY) segments of Bseg envs each form one contraction (env b = seg * Bseg + b'):
// the K unrolled uses of one latent conv reduce in a single launch (learner._flush_wgrad)
constexpr int WG_MAXSEG = 8;
struct WgImg {
  int B, H, W, Cin, Cout, E, KS, XR, stages_per_split;
  int Bseg;
  const bf16_t* xs[WG_MAXSEG];
  const bf16_t* dys[WG_MAXSEG];
};

MZ_DEV bf16x8_t tr_frag_at(const bf16_t* lo_base, const bf16_t* hi_base) {
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(lo_base));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(hi_base));
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

// 8 waves: waves 4 tg .. 4 tg + 3 own taps [5 tg, min(9, 5 tg + 5)) of the tile (two waves per
// SIMD to hide the LDS read latency; the tap groups write disjoint partials, so no reduction)
constexpr int WI_NT = 512;
constexpr int WI_PFN = WI_PF * 256 / WI_NT;  // staging chunks per thread
constexpr size_t WI_LDS_MAX = 140 * 1024;     // dynamic LDS (+ 16 KB static bias scratch <= 160 KB)
template <bool PF>
__global__ __launch_bounds__(WI_NT) void conv_wgrad_img_kernel(WgImg a, float* __restrict__ part,
                                                               float* __restrict__ bpart) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds_img[];
  bf16_t* ldy = lds_img;                                   // [KS][WI_LD]
  bf16_t* lx = lds_img + (size_t)(a.KS + WI_LEAD) * WI_LD;  // [XR + 64][WI_LD], preceded by WI_LEAD zero rows
  __shared__ float bred[WI_NT / 8][64];
  const int H = a.H, W = a.W, Wp = W + 2, Hp = H + 2, HWp = H * Wp, HpWp = Hp * Wp;
  const int nci = (a.Cin + 63) / 64;
  const int cit = blockIdx.x % nci, cot = blockIdx.x / nci;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tg = wave >> 2, wr = (wave >> 1) & 1, wc = wave & 1;
  const int tap0 = 5 * tg, ntap = tg ? 4 : 5;
  const int ch = tid & 7;  // 16-B chunk (8 channels) every staging chunk of this thread holds
  const int co_s = cot * 64 + ch * 8, ci_s = cit * 64 + ch * 8;
  const bool do_bias = bpart && cit == 0;
  float bacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bacc[j] = 0.f;
  // zero the lead rows and the tail margin of the X region once
  for (int i = tid; i < WI_LEAD * 8; i += WI_NT)
    *reinterpret_cast<uint4*>(lds_img + (size_t)(a.KS + i / 8) * WI_LD + (i & 7) * 8) = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < 64 * 8; i += WI_NT)
    *reinterpret_cast<uint4*>(lx + (size_t)(a.XR + i / 8) * WI_LD + (i & 7) * 8) = make_uint4(0, 0, 0, 0);
  f32x4_t acc[5][2][2];
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int nst_total = (a.B + a.E - 1) / a.E;
  const int st0 = blockIdx.y * a.stages_per_split, st1 = min(nst_total, st0 + a.stages_per_split);
  // stage staging through registers. PF: the next stage's HBM loads are in flight during this
  // stage's MFMAs (WI_PF chunks of 16 B per thread cover KS + XR rows x 8 chunks); otherwise the
  // stage is loaded in batches of WI_PF chunks after the previous one is consumed.
  // A stage = E consecutive envs of one segment (the planner makes E divide Bseg), so a chunk's
  // source is the stage's env-0 base + an offset that is the same for every stage: the per-chunk
  // index math (divisions by the bordered geometry) runs once per thread, not once per stage.
  const int nchunk = (a.KS + a.XR) * 8;
  const size_t img_x = (size_t)H * W * a.Cin, img_dy = (size_t)H * W * a.Cout;
  int soff[WI_PFN];     // element offset from the stage's env-0 base, -1 = zero chunk
  uint32_t sdy = 0u;    // bit u: chunk u is a dY chunk
  for (int u = 0; u < WI_PFN; ++u) {
    int off = -1;
    const int i = u * WI_NT + tid;
    if (i < a.KS * 8) {  // dY rows: k = e*HWp + y*Wp + xp (xp in 1..W real, 0 / W+1 border)
      const int r = i >> 3;
      const int e = r / HWp, w = r - e * HWp, y = w / Wp, xp = w - y * Wp;
      if (e < a.E && xp >= 1 && xp <= W && co_s < a.Cout) off = (int)(e * img_dy + (size_t)(y * W + xp - 1) * a.Cout + co_s);
      sdy |= 1u << u;
    } else if (i < nchunk) {  // X rows: bordered images, row e*HpWp + yp*Wp + xp
      const int r = (i >> 3) - a.KS;
      const int e = r / HpWp, rem = r - e * HpWp, yp = rem / Wp, xp = rem - yp * Wp;
      if (yp >= 1 && yp <= H && xp >= 1 && xp <= W && ci_s < a.Cin)
        off = (int)(e * img_x + (size_t)((yp - 1) * W + xp - 1) * a.Cin + ci_s);
    }
    soff[u] = off;
  }
  uint4 pf[WI_PFN];
  auto load_chunks = [&](int st, int base) {
    const int b0 = st * a.E, sg = b0 / a.Bseg, bl = b0 - sg * a.Bseg;
    const bf16_t* xb = a.xs[sg] + (size_t)bl * img_x;
    const bf16_t* db = a.dys[sg] + (size_t)bl * img_dy;
    if (base == 0) {
      // unconditional loads (zero chunks read the stage base, then select): a load under a
      // branch is waited for inside the branch, which serialised the 12 loads of a stage
#pragma unroll
      for (int u = 0; u < WI_PFN; ++u)
        pf[u] = *reinterpret_cast<const uint4*>(((sdy >> u) & 1u ? db : xb) + (soff[u] >= 0 ? soff[u] : 0));
#pragma unroll
      for (int u = 0; u < WI_PFN; ++u)
        if (soff[u] < 0) pf[u] = make_uint4(0, 0, 0, 0);
      return;
    }
#pragma unroll
    for (int u = 0; u < WI_PFN; ++u) {  // batched (non-PF) plans: chunks beyond the first batch
      const int i = base + u * WI_NT + tid;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (i < a.KS * 8) {
        const int r = i >> 3;
        const int e = r / HWp, w = r - e * HWp, y = w / Wp, xp = w - y * Wp;
        if (e < a.E && xp >= 1 && xp <= W && co_s < a.Cout)
          v = *reinterpret_cast<const uint4*>(db + e * img_dy + (size_t)(y * W + xp - 1) * a.Cout + co_s);
      } else if (i < nchunk) {
        const int r = (i >> 3) - a.KS;
        const int e = r / HpWp, rem = r - e * HpWp, yp = rem / Wp, xp = rem - yp * Wp;
        if (yp >= 1 && yp <= H && xp >= 1 && xp <= W && ci_s < a.Cin)
          v = *reinterpret_cast<const uint4*>(xb + e * img_x + (size_t)((yp - 1) * W + xp - 1) * a.Cin + ci_s);
      }
      pf[u] = v;
    }
  };
  auto store_chunks = [&](int base) {
#pragma unroll
    for (int u = 0; u < WI_PFN; ++u) {
      const int i = base + u * WI_NT + tid;
      if (i < a.KS * 8) {
        *reinterpret_cast<uint4*>(ldy + (size_t)(i >> 3) * WI_LD + ch * 8) = pf[u];
        if (do_bias) {
          const bf16_t* h = reinterpret_cast<const bf16_t*>(&pf[u]);
#pragma unroll
          for (int j = 0; j < 8; ++j) bacc[j] += bf16_to_f32(h[j]);
        }
      } else if (i < nchunk) {
        *reinterpret_cast<uint4*>(lx + (size_t)((i >> 3) - a.KS) * WI_LD + ch * 8) = pf[u];
      }
    }
  };
  if (PF && st0 < st1) load_chunks(st0, 0);
  for (int st = st0; st < st1; ++st) {
    __syncthreads();  // previous stage fully consumed
    if (PF) {
      store_chunks(0);
    } else {
      for (int base = 0; base < nchunk; base += WI_PFN * WI_NT) {
        load_chunks(st, base);
        store_chunks(base);
      }
    }
    __syncthreads();
    if (PF && st + 1 < st1) load_chunks(st + 1, 0);
    for (int ks = 0; ks < a.KS / 32; ++ks) {
      // this lane's transposed-read rows for the two 4-row blocks of k step ks
      const int r0 = ks * 32 + 4 * g + q, r1 = r0 + 16;
      const int e0 = min(r0 / HWp, a.E - 1), e1 = min(r1 / HWp, a.E - 1);
      const int x0 = e0 * HpWp + Wp + (r0 - e0 * HWp), x1 = e1 * HpWp + Wp + (r1 - e1 * HWp);
      bf16x8_t af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = wr * 32 + i * 16 + 4 * pp;
        af[i] = tr_frag_at(ldy + (size_t)r0 * WI_LD + c, ldy + (size_t)r1 * WI_LD + c);
      }
      // B fragments one tap ahead: tap t + 1's transposed reads are in flight during tap t's MFMAs
      auto bload = [&](int t, bf16x8_t (&b)[2]) {
        const int off = (t / 3 - 1) * Wp + (t % 3 - 1);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = wc * 32 + j * 16 + 4 * pp;
          b[j] = tr_frag_at(lx + (ptrdiff_t)(x0 + off) * WI_LD + c, lx + (ptrdiff_t)(x1 + off) * WI_LD + c);
        }
      };
      bf16x8_t bcur[2], bnxt[2];
      bload(tap0, bcur);
#pragma unroll
      for (int tt = 0; tt < 5; ++tt) {
        if (tt < ntap) {  // wave-uniform: tap group 1 has 4 taps
          if (tt + 1 < ntap) bload(tap0 + tt + 1, bnxt);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[tt][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bcur[j], acc[tt][i][j], 0, 0, 0);
          if (tt + 1 < ntap) { bcur[0] = bnxt[0]; bcur[1] = bnxt[1]; }
        }
      }
    }
  }
  const size_t K = (size_t)9 * a.Cin;
  float* outp = part + (size_t)blockIdx.y * a.Cout * K;
  const int fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int tt = 0; tt < 5; ++tt)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int t = tap0 + tt;
        const int ci = cit * 64 + wc * 32 + j * 16 + fr;
        if (tt >= ntap) continue;
        if (ci >= a.Cin) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = cot * 64 + wr * 32 + i * 16 + 4 * fk + r;
          if (co < a.Cout) outp[(size_t)co * K + (size_t)t * a.Cin + ci] = acc[tt][i][j][r];
        }
      }
  if (do_bias) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) bred[tid >> 3][ch * 8 + j] = bacc[j];
    __syncthreads();
    if (tid < 64) {
      float sum = 0.f;
      for (int r = 0; r < WI_NT / 8; ++r) sum += bred[r][tid];
      const int co = cot * 64 + tid;
      if (co < a.Cout) bpart[(size_t)blockIdx.y * a.Cout + co] = sum;
    }
  }
}

// geometry of the image-stage weight gradient (E envs per stage within the LDS budget)
struct WgPlan {
  WgImg a;
  int nsplit;
  size_t lds;
  bool pf;  // the whole stage fits the register prefetch
};
// B = all envs (nseg * Bseg); a stage's E envs never straddle a segment (E divides Bseg)
static bool wgrad_img_plan(int B, int Bseg, int H, int W, int Cin, int Cout, WgPlan& p) {
  const int Wp = W + 2, HWp = H * Wp, HpWp = (H + 2) * Wp;
  if (HWp % 4 || Bseg <= 0 || B % Bseg) return false;
  int E = 1;
  auto rows = [&](int e) { return ((e * HWp + 31) / 32 * 32) + WI_LEAD + e * HpWp + 64; };
  auto staged = [&](int e) { return (e * HWp + 31) / 32 * 32 + e * HpWp; };
  while (E < 16 && Bseg % (E * 2) == 0 && (size_t)rows(E * 2) * WI_LD * 2 <= WI_LDS_MAX && staged(E * 2) * 8 <= WI_PF * 256) E *= 2;
  if ((size_t)rows(E) * WI_LD * 2 > WI_LDS_MAX) return false;
  p.pf = staged(E) * 8 <= WI_PF * 256;
  const int tiles = ((Cout + 63) / 64) * ((Cin + 63) / 64);
  const int stages = (B + E - 1) / E;
  // one workgroup per CU (two per CU measured slower: the extra split partials cost more)
  int nsplit = (256 + tiles - 1) / tiles;
  if (nsplit > stages) nsplit = stages;
  const int sps = (stages + nsplit - 1) / nsplit;
  nsplit = (stages + sps - 1) / sps;
  p.a = WgImg{B, H, W, Cin, Cout, E, (E * HWp + 31) / 32 * 32, E * HpWp, sps, Bseg, {}, {}};
  p.nsplit = nsplit;
  p.lds = (size_t)rows(E) * WI_LD * 2;
  return true;
}

// bf16 3x3 weight gradient over pixel rows (round 6): the whole-image kernel's tiling (64 co x 64 ci,
// all 9 taps, 8 waves) without the zero border. The contraction index k runs over the E * HW real
// pixels of a stage — row e * HW + p of dY and of X, which is how E consecutive envs already lie in
// HBM — padded to a multiple of 32 with zero dY rows. Tap (dy, dx) of k row r is X row r + dy * W + dx,
// or the zero row XR where the tap leaves the image: each lane hands its own row address to the
// transposed read, with the 9-tap validity of its two k rows from a per-workgroup mask table (the same
// for every stage). Against the bordered kernel: 20 instead of 28 k per 4x5 image (the border columns'
// MFMAs and staging rows are gone), twice the envs per stage (10 k steps between barriers instead of 7),
// no per-step divisions, and an XCD-aware workgroup order (the 16 tiles of one env range share an L2).
struct WgPx {
  int B, H, W, Cin, Cout, E, KS, XR, stages_per_split, Bseg, tiles, remap;
  const bf16_t* xs[WG_MAXSEG];
  const bf16_t* dys[WG_MAXSEG];
};

// WF (the waves' share of the 64 x 64 x 9 tile; 2 = WF 1 with its k steps software-pipelined): 0 = 32 co x
// 32 ci x 5 / 4 taps per wave (2 A + 10 B fragment
// reads per 20 MFMAs); 1 = 64 co x 32 ci x 3 / 2 taps per wave (taps {0,1,2}, {3,4}, {5,6}, {7,8}; 4 A + 6 / 4 B
// reads per 24 / 16 MFMAs: 29 % fewer LDS fragment reads per stage). A SIMD holds waves w and w + 4, so each
// SIMD runs one 3-tap and one 2-tap wave (40 MFMAs per k step, as WF 0) or two 2-tap waves. Every output
// element is the same chain of the same MFMAs over the same fragments in both forms: the same bits.
template <int WF>
__global__ __launch_bounds__(WI_NT) void conv_wgrad_px_kernel(WgPx a, float* __restrict__ part,
                                                              float* __restrict__ bpart) {
  constexpr int NT = WF ? 3 : 5, NI = WF ? 4 : 2;  // taps and 16-row co fragments per wave
  extern __shared__ __attribute__((aligned(16))) bf16_t lds_img[];
  bf16_t* ldy = lds_img;                                      // [KS][WI_LD]
  bf16_t* lx = lds_img + (size_t)a.KS * WI_LD;                // [XR + 1][WI_LD], row XR = zeros
  uint16_t* tmask = reinterpret_cast<uint16_t*>(lx + (size_t)(a.XR + 1) * WI_LD);  // [KS]
  __shared__ float bred[WI_NT / 8][64];
  const int H = a.H, W = a.W, HW = H * W, NR = a.E * HW;
  const int nci = (a.Cin + 63) / 64;
  // workgroup -> (tile, split). remap: workgroup ids congruent mod 8 run on one XCD; they take
  // consecutive split-major work items, so the tiles of one env range read its X / dY through one L2
  int tile = blockIdx.x, split = blockIdx.y;
  if (a.remap) {
    const int L = blockIdx.x + blockIdx.y * gridDim.x, per = (gridDim.x * gridDim.y) >> 3;
    const int Lp = (L & 7) * per + (L >> 3);
    tile = Lp % a.tiles;
    split = Lp / a.tiles;
  }
  const int cit = tile % nci, cot = tile / nci;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave & 1;
  const int tg = WF ? wave >> 1 : wave >> 2, wr = WF ? 0 : (wave >> 1) & 1;
  const int tap0 = WF ? (tg ? 2 * tg + 1 : 0) : 5 * tg, ntap = WF ? (tg ? 2 : 3) : (tg ? 4 : 5);
  const int ch = tid & 7;
  const int co_s = cot * 64 + ch * 8, ci_s = cit * 64 + ch * 8;
  const bool do_bias = bpart && cit == 0;
  float bacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bacc[j] = 0.f;
  if (tid < 8) *reinterpret_cast<uint4*>(lx + (size_t)a.XR * WI_LD + tid * 8) = make_uint4(0, 0, 0, 0);
  for (int r = tid; r < a.KS; r += WI_NT) {  // bit t: tap t of pixel row r stays inside its image
    uint32_t m = 0u;
    if (r < NR) {
      const int p = r % HW, y = p / W, x = p - (p / W) * W;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int sy = y + t / 3 - 1, sx = x + t % 3 - 1;
        if (sy >= 0 && sy < H && sx >= 0 && sx < W) m |= 1u << t;
      }
    }
    tmask[r] = (uint16_t)m;
  }
  f32x4_t acc[NT][NI][2];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int nst_total = a.B / a.E;
  const int st0 = split * a.stages_per_split, st1 = min(nst_total, st0 + a.stages_per_split);
  // every chunk of a stage in one register batch (the planner guarantees (KS + XR) * 8 <= WI_PFN * WI_NT):
  // the next stage's loads are in flight during this stage's MFMAs. Offsets from the stage's env-0 base
  // are the same for every stage.
  const int nchunk = (a.KS + a.XR) * 8;
  // chunk u of a stage: offset from the stage's env-0 base, -1 for a zero chunk (WF 1 recomputes it per stage
  // instead of holding WI_PFN offsets in registers beside its larger accumulator set)
  auto chunk_off = [&](int u) {
    int off = -1;
    const int i = u * WI_NT + tid;
    if (i < a.KS * 8) {
      const int r = i >> 3;
      if (r < NR && co_s < a.Cout) off = r * a.Cout + co_s;
    } else if (i < nchunk) {
      const int r = (i >> 3) - a.KS;
      if (ci_s < a.Cin) off = r * a.Cin + ci_s;
    }
    return off;
  };
  int soff[WF ? 1 : WI_PFN];
  if constexpr (!WF) {
#pragma unroll
    for (int u = 0; u < WI_PFN; ++u) soff[u] = chunk_off(u);
  }
  uint4 pf[WI_PFN];
  auto load_stage = [&](int st) {
    const int b0 = st * a.E, sg = b0 / a.Bseg, bl = b0 - sg * a.Bseg;
    const bf16_t* xb = a.xs[sg] + (size_t)bl * HW * a.Cin;
    const bf16_t* db = a.dys[sg] + (size_t)bl * HW * a.Cout;
    int offs[WI_PFN];
#pragma unroll
    for (int u = 0; u < WI_PFN; ++u) {
      if constexpr (WF) offs[u] = chunk_off(u);
      else offs[u] = soff[u];
    }
#pragma unroll
    for (int u = 0; u < WI_PFN; ++u)
      pf[u] = *reinterpret_cast<const uint4*>((u * WI_NT + tid < a.KS * 8 ? db : xb) + (offs[u] >= 0 ? offs[u] : 0));
#pragma unroll
    for (int u = 0; u < WI_PFN; ++u)
      if (offs[u] < 0) pf[u] = make_uint4(0, 0, 0, 0);
  };
  auto store_stage = [&]() {
#pragma unroll
    for (int u = 0; u < WI_PFN; ++u) {
      const int i = u * WI_NT + tid;
      if (i < a.KS * 8) {
        *reinterpret_cast<uint4*>(ldy + (size_t)(i >> 3) * WI_LD + ch * 8) = pf[u];
        if (do_bias) {
          const bf16_t* h = reinterpret_cast<const bf16_t*>(&pf[u]);
#pragma unroll
          for (int j = 0; j < 8; ++j) bacc[j] += bf16_to_f32(h[j]);
        }
      } else if (i < nchunk) {
        *reinterpret_cast<uint4*>(lx + (size_t)((i >> 3) - a.KS) * WI_LD + ch * 8) = pf[u];
      }
    }
  };
  if (st0 < st1) load_stage(st0);
  for (int st = st0; st < st1; ++st) {
    __syncthreads();  // previous stage fully consumed (first pass: the zero row and mask table written)
    store_stage();
    __syncthreads();
#ifndef MZBA_WGRAD_ABLATE
#define MZBA_WGRAD_ABLATE 0  // diagnostic builds only (numerically wrong): 1 no next-stage loads, 3 no B-tap reloads
#endif
    if (MZBA_WGRAD_ABLATE != 1 && st + 1 < st1) load_stage(st + 1);
    if constexpr (WF == 2) {
      // the k steps software-pipelined: the last tap's MFMAs of step ks interleave the A fragments and the
      // first tap's B fragments of step ks + 1 (each register refilled right after the last MFMA reading it),
      // so a step no longer opens on a full LDS round trip. The same MFMAs in the same order per element.
      const int nks = a.KS / 32;
      int r0 = 4 * g + q, r1 = r0 + 16;
      uint32_t m0 = tmask[r0], m1 = tmask[r1];
      auto afrag = [&](int i, int s0, int s1) {
        const int c = i * 16 + 4 * pp;
        return tr_frag_at(ldy + (size_t)s0 * WI_LD + c, ldy + (size_t)s1 * WI_LD + c);
      };
      auto bload = [&](int t, int s0, int s1, uint32_t k0, uint32_t k1, bf16x8_t (&b)[2]) {
        const int off = (t / 3 - 1) * W + (t % 3 - 1);
        const int x0 = (k0 >> t) & 1u ? s0 + off : a.XR, x1 = (k1 >> t) & 1u ? s1 + off : a.XR;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = wc * 32 + j * 16 + 4 * pp;
          b[j] = tr_frag_at(lx + (size_t)x0 * WI_LD + c, lx + (size_t)x1 * WI_LD + c);
        }
      };
      bf16x8_t af[NI], bcur[2], bnxt[2];
#pragma unroll
      for (int i = 0; i < NI; ++i) af[i] = afrag(i, r0, r1);
      bload(tap0, r0, r1, m0, m1, bcur);
      for (int ks = 0; ks < nks; ++ks) {
        // the last step re-reads its own rows (valid addresses, results unused): no branches in the loop
        const int step = ks + 1 < nks ? 32 : 0;
        const int n0 = r0 + step, n1 = r1 + step;
        const uint32_t nm0 = tmask[n0], nm1 = tmask[n1];
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          if (tt < ntap) {  // wave-uniform
            if (tt + 1 < ntap) {
              bload(tap0 + tt + 1, r0, r1, m0, m1, bnxt);
#pragma unroll
              for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                  acc[tt][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bcur[j], acc[tt][i][j], 0, 0, 0);
              bcur[0] = bnxt[0];
              bcur[1] = bnxt[1];
            } else {
#pragma unroll
              for (int i = 0; i < NI; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
                  acc[tt][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bcur[j], acc[tt][i][j], 0, 0, 0);
                af[i] = afrag(i, n0, n1);
              }
              bload(tap0, n0, n1, nm0, nm1, bcur);
            }
          }
        }
        r0 = n0;
        r1 = n1;
        m0 = nm0;
        m1 = nm1;
      }
    } else {
      for (int ks = 0; ks < a.KS / 32; ++ks) {
        const int r0 = ks * 32 + 4 * g + q, r1 = r0 + 16;
        const uint32_t m0 = tmask[r0], m1 = tmask[r1];
        bf16x8_t af[NI];
  #pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int c = wr * 32 + i * 16 + 4 * pp;
          af[i] = tr_frag_at(ldy + (size_t)r0 * WI_LD + c, ldy + (size_t)r1 * WI_LD + c);
        }
        auto bload = [&](int t, bf16x8_t (&b)[2]) {
          const int off = (t / 3 - 1) * W + (t % 3 - 1);
          const int x0 = (m0 >> t) & 1u ? r0 + off : a.XR, x1 = (m1 >> t) & 1u ? r1 + off : a.XR;
  #pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int c = wc * 32 + j * 16 + 4 * pp;
            b[j] = tr_frag_at(lx + (size_t)x0 * WI_LD + c, lx + (size_t)x1 * WI_LD + c);
          }
        };
        bf16x8_t bcur[2], bnxt[2];
        bload(tap0, bcur);
  #pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          if (tt < ntap) {  // wave-uniform: the last tap group(s) have one tap fewer
            if (tt + 1 < ntap) {
            if (MZBA_WGRAD_ABLATE == 3) { bnxt[0] = bcur[0]; bnxt[1] = bcur[1]; }
            else bload(tap0 + tt + 1, bnxt);
          }
  #pragma unroll
            for (int i = 0; i < NI; ++i)
  #pragma unroll
              for (int j = 0; j < 2; ++j)
                acc[tt][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bcur[j], acc[tt][i][j], 0, 0, 0);
            if (tt + 1 < ntap) { bcur[0] = bnxt[0]; bcur[1] = bnxt[1]; }
          }
        }
      }
    }
  }
  const size_t K = (size_t)9 * a.Cin;
  float* outp = part + (size_t)split * a.Cout * K;
  const int fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int t = tap0 + tt;
        const int ci = cit * 64 + wc * 32 + j * 16 + fr;
        if (tt >= ntap) continue;
        if (ci >= a.Cin) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = cot * 64 + wr * 32 + i * 16 + 4 * fk + r;
          if (co < a.Cout) outp[(size_t)co * K + (size_t)t * a.Cin + ci] = acc[tt][i][j][r];
        }
      }
  if (do_bias) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) bred[tid >> 3][ch * 8 + j] = bacc[j];
    __syncthreads();
    if (tid < 64) {
      float sum = 0.f;
      for (int r = 0; r < WI_NT / 8; ++r) sum += bred[r][tid];
      const int co = cot * 64 + tid;
      if (co < a.Cout) bpart[(size_t)split * a.Cout + co] = sum;
    }
  }
}

struct WgPxPlan {
  WgPx a;
  int nsplit;
  size_t lds;
};
// B = all envs (nseg * Bseg); E (envs per stage) divides Bseg, so a stage never straddles a segment and
// every stage is full; false when one env's stage does not fit the register batch or the LDS budget
static bool wgrad_px_plan(int B, int Bseg, int H, int W, int Cin, int Cout, WgPxPlan& p) {
  const int HW = H * W;
  if (HW <= 0 || Bseg <= 0 || B % Bseg) return false;
  auto ksr = [&](int e) { return (e * HW + 31) / 32 * 32; };
  auto bytes = [&](int e) { return (size_t)(ksr(e) + e * HW + 1) * WI_LD * 2 + (size_t)ksr(e) * 2; };
  auto fits = [&](int e) { return bytes(e) <= WI_LDS_MAX && (ksr(e) + e * HW) * 8 <= WI_PFN * WI_NT; };
  if (!fits(1)) return false;
  int E = 1;
  while (E < 64 && Bseg % (E * 2) == 0 && fits(E * 2)) E *= 2;
  const int tiles = ((Cout + 63) / 64) * ((Cin + 63) / 64);
  const int stages = B / E;
  int nsplit = (256 + tiles - 1) / tiles;  // one workgroup per CU
  if (nsplit > stages) nsplit = stages;
  const int sps = (stages + nsplit - 1) / nsplit;
  nsplit = (stages + sps - 1) / sps;
  p.a = WgPx{B, H, W, Cin, Cout, E, ksr(E), E * HW, sps, Bseg, tiles, (tiles * nsplit) % 8 == 0, {}, {}};
  p.nsplit = nsplit;
  p.lds = bytes(E);
  return true;
}

// the weight and bias partials of one split weight-gradient launch, summed in one launch: acc[i] += sum_s
// part[s][i] for i < n, bacc[j] += sum_s bpart[s][j] for j < nb, each element in split order (round 4: one launch
// instead of one per buffer, the same sums)
constexpr int SP_FK = 16;
__global__ void sum_partials2_kernel(const float* __restrict__ part, const float* __restrict__ bpart, int nsplit,
                                     size_t n, size_t nb, float* __restrict__ acc, float* __restrict__ bacc) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n + nb; i += (size_t)gridDim.x * blockDim.x) {
    const bool w = i < n;
    const float* p = w ? part + i : bpart + (i - n);
    const size_t st = w ? n : nb;
    // the first SP_FK partials loaded before the first add (a rolled loop waited one round trip per split); the
    // adds keep split order
    float* dst = w ? acc + i : bacc + (i - n);
    const float a0 = *dst;  // loaded with the partials (read after the sum it was one more round trip)
    float v[SP_FK];
#pragma unroll
    for (int k = 0; k < SP_FK; ++k) v[k] = k < nsplit ? p[(size_t)k * st] : 0.f;
    float s = v[0];
#pragma unroll
    for (int k = 1; k < SP_FK; ++k)
      if (k < nsplit) s += v[k];
    for (int k = SP_FK; k < nsplit; ++k) s += p[(size_t)k * st];
    *dst = a0 + s;
  }
}

// ------------------------------------------------------------------ avg-pool backward, axpy
template <typename T>
__global__ void avgpool2_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int B, int H, int W, int C) {
  const size_t n = (size_t)B * H * W * C;
  const int Ho = H / 2, Wo = W / 2;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    size_t q = i / C;
    const int xx = (int)(q % W); q /= W;
    const int yy = (int)(q % H);
    const size_t b = q / H;
    st(dx + i, ld(dy + ((b * Ho + yy / 2) * Wo + xx / 2) * C + c) / 4.0f);
  }
}

// the same element values, 4 channels per thread (C % 4 == 0) with 32-bit index arithmetic (n < 2^31): the
// per-element 64-bit divisions above held the kernel at a fifth of the HBM rate
template <typename T>
__global__ void avgpool2_bwd4_kernel(const T* __restrict__ dy, T* __restrict__ dx, int B, int H, int W, int C) {
  const int C4 = C / 4, Ho = H / 2, Wo = W / 2;
  const unsigned n4 = (unsigned)B * H * W * C4;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const unsigned c4 = i % C4;
    unsigned q = i / C4;
    const unsigned xx = q % W;
    q /= W;
    const unsigned yy = q % H, b = q / H;
    const float4 v = Vec4<T>::load(dy + ((size_t)(b * Ho + yy / 2) * Wo + xx / 2) * C + 4 * c4);
    Vec4<T>::store(dx + (size_t)i * 4, make_float4(v.x / 4.0f, v.y / 4.0f, v.z / 4.0f, v.w / 4.0f));
  }
}

template <typename T>
__global__ void axpy_kernel(T* __restrict__ y, const T* __restrict__ x, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    st(y + i, ld(y + i) + ld(x + i));
}

// ------------------------------------------------------------------ min-max scale
// one workgroup per env over n = HW*C values (NHWC); the first min / max in NCHW order
// (index c*HW + p) is recorded for the backward. mm[b] = (min, max), idx[b] = NHWC indices.
template <typename T>
__global__ __launch_bounds__(256) void scale_fwd_kernel(const T* __restrict__ h, T* __restrict__ out,
                                                        float2* __restrict__ mm, int2* __restrict__ idx, int HW,
                                                        int C) {
  const int b = blockIdx.x, n = HW * C;
  const T* x = h + (size_t)b * n;
  float mn = INFINITY, mx = -INFINITY;
  int kmn = 0x7fffffff, kmx = 0x7fffffff;  // NCHW keys
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = ld(x + i);
    const int c = i % C, key = c * HW + i / C;
    if (v < mn || (v == mn && key < kmn)) { mn = v; kmn = key; }
    if (v > mx || (v == mx && key < kmx)) { mx = v; kmx = key; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(mn, o), x2 = __shfl_xor(mx, o);
    const int k2 = __shfl_xor(kmn, o), kx2 = __shfl_xor(kmx, o);
    if (m2 < mn || (m2 == mn && k2 < kmn)) { mn = m2; kmn = k2; }
    if (x2 > mx || (x2 == mx && kx2 < kmx)) { mx = x2; kmx = kx2; }
  }
  __shared__ float smn[4], smx[4];
  __shared__ int skn[4], skx[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smn[w] = mn; smx[w] = mx; skn[w] = kmn; skx[w] = kmx; }
  __syncthreads();
  mn = smn[0]; mx = smx[0]; kmn = skn[0]; kmx = skx[0];
  for (int k = 1; k < 4; ++k) {
    if (smn[k] < mn || (smn[k] == mn && skn[k] < kmn)) { mn = smn[k]; kmn = skn[k]; }
    if (smx[k] > mx || (smx[k] == mx && skx[k] < kmx)) { mx = smx[k]; kmx = skx[k]; }
  }
  const float den = (mx - mn) + 1e-8f;
  T* o = out + (size_t)b * n;
  for (int i = threadIdx.x; i < n; i += 256) st(o + i, (ld(x + i) - mn) / den);
  if (threadIdx.x == 0) {
    mm[b] = make_float2(mn, mx);
    idx[b] = make_int2((kmn % HW) * C + kmn / HW, (kmx % HW) * C + kmx / HW);
  }
}

// dh (=|+=) dy/den, then dh[argmin] += -sum(dy)/den - d_den, dh[argmax] += d_den with
// d_den = -sum(dy * (h - min)) / den^2 (autograd of (h - min) / (max - min + 1e-8))
template <typename T>
__global__ __launch_bounds__(256) void scale_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ h,
                                                        const float2* __restrict__ mm, const int2* __restrict__ idx,
                                                        T* dh, int n, int accumulate) {
  const int b = blockIdx.x;
  const float mn = mm[b].x, mx = mm[b].y;
  const float den = (mx - mn) + 1e-8f;
  const T* g = dy + (size_t)b * n;
  const T* x = h + (size_t)b * n;
  T* o = dh + (size_t)b * n;
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float gv = ld(g + i);
    const float d = gv / den;
    s1 += d;
    s2 += gv * (ld(x + i) - mn);
    st(o + i, accumulate ? ld(o + i) + d : d);
  }
  for (int off = 32; off > 0; off >>= 1) { s1 += __shfl_xor(s1, off); s2 += __shfl_xor(s2, off); }
  __shared__ float r1[4], r2[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { r1[w] = s1; r2[w] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float S1 = (r1[0] + r1[1]) + (r1[2] + r1[3]);
    const float S2 = (r2[0] + r2[1]) + (r2[2] + r2[3]);
    const float dden = -(S2 / den) / den;
    const int2 k = idx[b];
    st(o + k.x, ld(o + k.x) + (-S1 - dden));
    st(o + k.y, ld(o + k.y) + dden);
  }
}

// ------------------------------------------------------------------ heads: nn.Linear on NHWC
// out[b][o] = bias[o] + sum_k w[o][k] x[b][k], k = p*C + c (weights kept in that order)
template <typename T>
__global__ __launch_bounds__(256) void linear_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ out,
                                                         int K, int O) {
  const int b = blockIdx.x;
  const T* xb = x + (size_t)b * K;
  float acc[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) acc[o] = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float v = ld(xb + k);
    float wv[16];  // unconditional loads (rows >= O re-read row 0): a load under `if (o < O)` is
#pragma unroll     // waited for inside its branch, which serialised the 16 loads
    for (int o = 0; o < 16; ++o) wv[o] = w[(size_t)(o < O ? o : 0) * K + k];
#pragma unroll
    for (int o = 0; o < 16; ++o)
      if (o < O) acc[o] += v * wv[o];
  }
  __shared__ float red[4][16];
  const int w_ = threadIdx.x >> 6;
#pragma unroll
  for (int o = 0; o < 16; ++o) {
    float v = acc[o];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) red[w_][o] = v;
  }
  __syncthreads();
  if (threadIdx.x < O) {
    const int o = threadIdx.x;
    out[(size_t)b * O + o] = ((red[0][o] + red[1][o]) + (red[2][o] + red[3][o])) + bias[o];
  }
}

// dx[b][k] (=|+=) sum_o dy[b][o] w[o][k]
template <typename T>
__global__ void linear_bwd_x_kernel(const float* __restrict__ dy, const float* __restrict__ w, T* dx, int B, int K,
                                    int O, int accumulate) {
  const size_t n = (size_t)B * K;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % K);
    const size_t b = i / K;
    float s = 0.f;
    for (int o = 0; o < O; ++o) s += dy[b * O + o] * w[(size_t)o * K + k];
    st(dx + i, accumulate ? ld(dx + i) + s : s);
  }
}

// part[split][o][k] = sum_{b in split} dy[b][o] x[b][k]; bpart[split][o] = sum dy[b][o]
template <typename T>
__global__ void linear_bwd_w_kernel(const float* __restrict__ dy, const T* __restrict__ x, int B, int K, int O,
                                    int rows_per_split, float* __restrict__ part, float* __restrict__ bpart) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int split = blockIdx.y;
  const int b0 = split * rows_per_split, b1 = min(B, b0 + rows_per_split);
  float acc[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) acc[o] = 0.f;
  if (k < K)
    for (int b = b0; b < b1; ++b) {
      const float v = ld(x + (size_t)b * K + k);
#pragma unroll
      for (int o = 0; o < 16; ++o)
        if (o < O) acc[o] += dy[(size_t)b * O + o] * v;
    }
  if (k < K)
    for (int o = 0; o < O; ++o) part[((size_t)split * O + o) * K + k] = acc[o];
  if (blockIdx.x == 0 && threadIdx.x < O) {
    float s = 0.f;
    for (int b = b0; b < b1; ++b) s += dy[(size_t)b * O + threadIdx.x];
    bpart[(size_t)split * O + threadIdx.x] = s;
  }
}

// ------------------------------------------------------------------ loss (loss_fn, train_torch.py:33-66)
// One workgroup. Row r = (b, k) of the (B, K) targets; logits[k][b][n]. Per row: compact
// transform + two-hot over the integer supports (utils.py:30-64), log_softmax, KL terms
// t*(log t - logp) (0 where t == 0), and the logit gradient (softmax*sum(t) - t)/(B*K)/K.
// loss[0..3] = total, reward, value, policy.
constexpr int LOSS_T = 256;

MZ_DEV void two_hot(float x, float smin, float smax, int ns, float* t) {
  const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
  const float c = sg * ((sqrtf(fabsf(x) + 1.f) - 1.f) + 0.001f * x);
  const float step = (smax - smin) / (float)(ns - 1);
  int lo = -1;  // searchsorted(right=True) - 1
  for (int i = 0; i < ns; ++i)
    if (smin + (float)i * step <= c) lo = i;
  lo = lo < 0 ? 0 : (lo > ns - 2 ? ns - 2 : lo);
  const float sl = smin + (float)lo * step, su = smin + (float)(lo + 1) * step;
  const float pl = (su - c) / ((su - sl) + 1e-10f);
  for (int i = 0; i < ns; ++i) t[i] = 0.f;
  t[lo] = pl;
  t[lo + 1] = 1.f - pl;
}

MZ_DEV double kl_row(const float* z, const float* t, int n, float scale, float* dz) {
  float m = z[0];
  for (int i = 1; i < n; ++i) m = fmaxf(m, z[i]);
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += expf(z[i] - m);
  const float ls = logf(s);
  float tsum = 0.f;
  double kl = 0.0;
  for (int i = 0; i < n; ++i) {
    const float lp = (z[i] - m) - ls;  // torch log_softmax: (x - max) - log(sum exp(x - max))
    if (t[i] > 0.f) kl += (double)(t[i] * (logf(t[i]) - lp));
    tsum += t[i];
  }
  for (int i = 0; i < n; ++i) dz[i] = (expf((z[i] - m) - ls) * tsum - t[i]) * scale;
  return kl;
}

__global__ __launch_bounds__(LOSS_T) void loss_kernel(const float* __restrict__ lr, const float* __restrict__ lv,
                                                      const float* __restrict__ lp, const float* __restrict__ rewards,
                                                      const float* __restrict__ targets,
                                                      const float* __restrict__ counts, const int32_t* slots, int B,
                                                      int K, int ns, int na, float smin, float smax,
                                                      float* __restrict__ dlr, float* __restrict__ dlv,
                                                      float* __restrict__ dlp, float* __restrict__ loss) {
  __shared__ double red[3][LOSS_T];
  const float scale = (1.f / (float)K) / (float)(B * K);
  double acc[3] = {0.0, 0.0, 0.0};
  for (int r = threadIdx.x; r < B * K; r += LOSS_T) {
    const int b = r / K, k = r - b * K;
    const size_t src = slots ? (size_t)slots[b] : (size_t)b;  // ring row of window b
    float t[16], z[16], dz[16];
    const size_t o1 = ((size_t)k * B + b) * ns, o3 = ((size_t)k * B + b) * na;
    two_hot(rewards[src * K + k], smin, smax, ns, t);
    for (int i = 0; i < ns; ++i) z[i] = lr[o1 + i];
    acc[0] += kl_row(z, t, ns, scale, dz);
    for (int i = 0; i < ns; ++i) dlr[o1 + i] = dz[i];
    two_hot(targets[src * K + k], smin, smax, ns, t);
    for (int i = 0; i < ns; ++i) z[i] = lv[o1 + i];
    acc[1] += kl_row(z, t, ns, scale, dz);
    for (int i = 0; i < ns; ++i) dlv[o1 + i] = dz[i];
    float cs = 0.f;
    for (int i = 0; i < na; ++i) cs += counts[(src * K + k) * na + i];
    for (int i = 0; i < na; ++i) { t[i] = counts[(src * K + k) * na + i] / cs; z[i] = lp[o3 + i]; }
    acc[2] += kl_row(z, t, na, scale, dz);
    for (int i = 0; i < na; ++i) dlp[o3 + i] = dz[i];
  }
  for (int j = 0; j < 3; ++j) red[j][threadIdx.x] = acc[j];
  __syncthreads();
  for (int s = LOSS_T / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int j = 0; j < 3; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float rl = (float)(red[0][0] / (B * K)), vl = (float)(red[1][0] / (B * K)), pl = (float)(red[2][0] / (B * K));
    loss[0] = (1.f / (float)K) * ((rl + vl) + pl);
    loss[1] = rl; loss[2] = vl; loss[3] = pl;
  }
}

// loss_kernel over many workgroups (round 5: the one-workgroup form took 159 us of the minibatch's critical path):
// a thread per row r computes its three KL terms (gradients written as loss_kernel) and stores them to
// ws[j][r]; loss_reduce_kernel then folds them exactly as loss_kernel's threads did — thread t adds rows t,
// t + LOSS_T, ... in order into its double accumulators, then the same tree — so the loss is bit-identical
__global__ __launch_bounds__(256) void loss_rows_kernel(const float* __restrict__ lr, const float* __restrict__ lv,
                                                        const float* __restrict__ lp, const float* __restrict__ rewards,
                                                        const float* __restrict__ targets,
                                                        const float* __restrict__ counts, const int32_t* slots, int B,
                                                        int K, int ns, int na, float smin, float smax,
                                                        float* __restrict__ dlr, float* __restrict__ dlv,
                                                        float* __restrict__ dlp, double* __restrict__ ws) {
  const float scale = (1.f / (float)K) / (float)(B * K);
  const int r = blockIdx.x * blockDim.x + threadIdx.x, BK = B * K;
  if (r >= BK) return;
  const int b = r / K, k = r - b * K;
  const size_t src = slots ? (size_t)slots[b] : (size_t)b;
  float t[16], z[16], dz[16];
  const size_t o1 = ((size_t)k * B + b) * ns, o3 = ((size_t)k * B + b) * na;
  two_hot(rewards[src * K + k], smin, smax, ns, t);
  for (int i = 0; i < ns; ++i) z[i] = lr[o1 + i];
  ws[r] = kl_row(z, t, ns, scale, dz);
  for (int i = 0; i < ns; ++i) dlr[o1 + i] = dz[i];
  two_hot(targets[src * K + k], smin, smax, ns, t);
  for (int i = 0; i < ns; ++i) z[i] = lv[o1 + i];
  ws[BK + r] = kl_row(z, t, ns, scale, dz);
  for (int i = 0; i < ns; ++i) dlv[o1 + i] = dz[i];
  float cs = 0.f;
  for (int i = 0; i < na; ++i) cs += counts[(src * K + k) * na + i];
  for (int i = 0; i < na; ++i) { t[i] = counts[(src * K + k) * na + i] / cs; z[i] = lp[o3 + i]; }
  ws[2 * BK + r] = kl_row(z, t, na, scale, dz);
  for (int i = 0; i < na; ++i) dlp[o3 + i] = dz[i];
}

__global__ __launch_bounds__(LOSS_T) void loss_reduce_kernel(const double* __restrict__ ws, int B, int K,
                                                             float* __restrict__ loss) {
  __shared__ double red[3][LOSS_T];
  const int BK = B * K;
  for (int j = 0; j < 3; ++j) {
    double acc = 0.0;
    int r = threadIdx.x;
    for (; r + 3 * LOSS_T < BK; r += 4 * LOSS_T) {  // four rows' loads ahead of their adds, added in row order
      const double v0 = ws[j * BK + r], v1 = ws[j * BK + r + LOSS_T], v2 = ws[j * BK + r + 2 * LOSS_T],
                   v3 = ws[j * BK + r + 3 * LOSS_T];
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; r < BK; r += LOSS_T) acc += ws[j * BK + r];
    red[j][threadIdx.x] = acc;
  }
  __syncthreads();
  for (int s = LOSS_T / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int j = 0; j < 3; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float rl = (float)(red[0][0] / (B * K)), vl = (float)(red[1][0] / (B * K)), pl = (float)(red[2][0] / (B * K));
    loss[0] = (1.f / (float)K) * ((rl + vl) + pl);
    loss[1] = rl; loss[2] = vl; loss[3] = pl;
  }
}

// ------------------------------------------------------------------ Adam (networks.py:268)
// g = grad + wd*p; m += (1-b1)(g - m); v = v*b2 + (1-b2)*g*g; p += (-step_size*m) / (sqrt(v)/bc2s + eps)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ grad, float* __restrict__ m,
                            float* __restrict__ v, size_t n, float neg_step, float one_m_b1, float b2, float one_m_b2,
                            float bc2s, float eps, float wd) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float pv = p[i];
    const float g = grad[i] + wd * pv;
    const float mv = m[i] + one_m_b1 * (g - m[i]);
    const float vv = v[i] * b2 + (one_m_b2 * g) * g;
    m[i] = mv;
    v[i] = vv;
    p[i] = pv + (neg_step * mv) / (sqrtf(vv) / bc2s + eps);
  }
}

// the same with the step-dependent scalars read from device memory (sc = {neg_step, 1-b1, b2, 1-b2,
// bc2s, eps, wd}): a captured minibatch graph replays with the host refreshing sc per step
__global__ void adam_dev_kernel(float* __restrict__ p, const float* __restrict__ grad, float* __restrict__ m,
                                float* __restrict__ v, size_t n, const float* __restrict__ sc) {
  const float neg_step = sc[0], one_m_b1 = sc[1], b2 = sc[2], one_m_b2 = sc[3], bc2s = sc[4], eps = sc[5], wd = sc[6];
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float pv = p[i];
    const float g = grad[i] + wd * pv;
    const float mv = m[i] + one_m_b1 * (g - m[i]);
    const float vv = v[i] * b2 + (one_m_b2 * g) * g;
    m[i] = mv;
    v[i] = vv;
    p[i] = pv + (neg_step * mv) / (sqrtf(vv) / bc2s + eps);
  }
}

// adam_kernel's / adam_dev_kernel's update, 4 parameters per thread (n % 4 == 0, 16-B aligned arrays: one 16-B access
// per array instead of four 4-B ones); DEV: the scalars from device memory (sc), else from the arguments
template <bool DEV>
__global__ void adam4_kernel(float4* __restrict__ p, const float4* __restrict__ grad, float4* __restrict__ m,
                             float4* __restrict__ v, size_t n4, const float* __restrict__ sc, float a_neg_step,
                             float a_one_m_b1, float a_b2, float a_one_m_b2, float a_bc2s, float a_eps, float a_wd) {
  const float neg_step = DEV ? sc[0] : a_neg_step, one_m_b1 = DEV ? sc[1] : a_one_m_b1, b2 = DEV ? sc[2] : a_b2;
  const float one_m_b2 = DEV ? sc[3] : a_one_m_b2, bc2s = DEV ? sc[4] : a_bc2s, eps = DEV ? sc[5] : a_eps;
  const float wd = DEV ? sc[6] : a_wd;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 p4 = p[i], g4 = grad[i], m4 = m[i], v4 = v[i];
    float po[4], mo[4], vo[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float pv = (&p4.x)[k];
      const float g = (&g4.x)[k] + wd * pv;
      const float mk = (&m4.x)[k];
      const float mv = mk + one_m_b1 * (g - mk);
      const float vv = (&v4.x)[k] * b2 + (one_m_b2 * g) * g;
      mo[k] = mv;
      vo[k] = vv;
      po[k] = pv + (neg_step * mv) / (sqrtf(vv) / bc2s + eps);
    }
    m[i] = make_float4(mo[0], mo[1], mo[2], mo[3]);
    v[i] = make_float4(vo[0], vo[1], vo[2], vo[3]);
    p[i] = make_float4(po[0], po[1], po[2], po[3]);
  }
}

// ------------------------------------------------------------------ learner inputs
// rep input [B][HW][Cp]: channel c < L = lut[frame code], L <= c < 2L = a/3 (train_torch.py:279-293,
// 437-470), zero beyond 2L. states u8 ring [cap][L][HW], past_actions i64 ring [cap][L].
template <typename T>
__global__ void learner_input_kernel(const uint8_t* __restrict__ states, const int64_t* __restrict__ past,
                                     const int32_t* __restrict__ slots, const float* __restrict__ lut, T* __restrict__ out,
                                     int B, int L, int HW, int Cp) {
  const size_t n = (size_t)B * HW * Cp;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const size_t q = i / Cp;
    const int p = (int)(q % HW);
    const size_t b = q / HW, s = (size_t)slots[b];
    float v = 0.f;
    if (c < L) v = lut[states[(s * L + c) * HW + p] & 7];
    else if (c < 2 * L) v = (float)past[s * L + (c - L)] / 3.0f;
    st(out + i, v);
  }
}

// dynamics input [B][HW][Cp] = [h (C channels), one-hot(a) (3), 0...] (train_torch.py:295-311)
template <typename T>
__global__ void dyn_input_kernel(const T* __restrict__ h, const int64_t* __restrict__ fut,
                                 const int32_t* __restrict__ slots, int K, int k, T* __restrict__ out, int B, int HW,
                                 int C, int A, int Cp) {
  const size_t n = (size_t)B * HW * Cp;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const size_t q = i / Cp;  // b*HW + p
    const size_t b = q / HW;
    float v = 0.f;
    if (c < C) v = ld(h + q * C + c);
    else if (c < C + A) v = (fut[(size_t)slots[b] * K + k] == (int64_t)(c - C)) ? 1.f : 0.f;
    st(out + i, v);
  }
}

unsigned grid_for(size_t n, int block = 256, unsigned cap = 16384) {
  size_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}

template <typename F>
int dispatch(int dtype, F&& f) {
  if (dtype == 0) return f(float{});
  if (dtype == 1) return f(bf16_t{});
  return -9;
}

}  // namespace

extern "C" {

int mzba_bn_stats(int dtype, const void* x, int M, int C, float eps, float momentum, const float* gamma,
                  const float* beta, float* stats, float* run_mean, float* run_var, void* ws, long long ws_bytes,
                  hipStream_t stream) {
  MZ_CHECK_ARG(x && stats && gamma && beta && ws && M > 0 && C > 0 && C % 4 == 0, -1);
  const int rpc = BN_RPC;
  const int nchunk = (M + rpc - 1) / rpc;
  MZ_CHECK_ARG((long long)nchunk * C * (long long)sizeof(float2) <= ws_bytes, -2);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(bn_stats_partial_kernel<T>, dim3((C + 63) / 64, nchunk), dim3(256), 0, stream, (const T*)x, M,
                       C, rpc, (float2*)ws);
    hipLaunchKernelGGL(bn_stats_final_kernel, dim3(C), dim3(64), 0, stream, (const float2*)ws, nchunk,
                       rpc, M, C, eps, momentum, gamma, beta, stats, run_mean, run_var);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_bn_stats_final(const float* part, int nchunk, int rpc, int M, int C, float eps, float momentum,
                        const float* gamma, const float* beta, float* stats, float* run_mean, float* run_var,
                        hipStream_t stream) {
  MZ_CHECK_ARG(part && stats && gamma && beta && nchunk > 0 && rpc > 0 && M > 0 && C > 0 &&
               (long long)nchunk * rpc >= M && (long long)(nchunk - 1) * rpc < M, -1);
  hipLaunchKernelGGL(bn_stats_final_kernel, dim3(C), dim3(64), 0, stream, (const float2*)part, nchunk, rpc, M, C, eps,
                     momentum, gamma, beta, stats, run_mean, run_var);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_bn_backward_final(int dtype, const void* g, const void* x, const float* stats, const float* part, int nchunk,
                           int M, int C, float* dgamma, float* dbeta, void* dx, void* ws, long long ws_bytes,
                           hipStream_t stream) {
  MZ_CHECK_ARG(g && x && stats && part && dgamma && dbeta && dx && ws && nchunk > 0 && M > 0 && C > 0 && C % 4 == 0,
               -1);
  MZ_CHECK_ARG(3LL * C * 4 <= ws_bytes, -2);
  float* coef = (float*)ws;
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(C), dim3(64), 0, stream, (const float2*)part, nchunk, M, C, stats,
                       dgamma, dbeta, coef);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(grid_for((size_t)M * C / 4)), dim3(256), 0, stream, (const T*)g,
                       (const T*)x, stats, (const float*)coef, (T*)dx, M, C);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_bn_backward_apply(int dtype, const void* g, const void* x, const float* stats, const float* coef, void* dx,
                           int M, int C, hipStream_t stream) {
  MZ_CHECK_ARG(g && x && stats && coef && dx && M > 0 && C > 0 && C % 4 == 0, -1);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(grid_for((size_t)M * C / 4)), dim3(256), 0, stream, (const T*)g,
                       (const T*)x, stats, coef, (T*)dx, M, C);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_bn_backward_coef(const float* part, int nchunk, int M, int C, const float* stats, float* dgamma, float* dbeta,
                          float* coef, hipStream_t stream) {
  MZ_CHECK_ARG(part && stats && dgamma && dbeta && coef && nchunk > 0 && M > 0 && C > 0, -1);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(C), dim3(64), 0, stream, (const float2*)part, nchunk, M, C, stats,
                     dgamma, dbeta, coef);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_bn_apply(int dtype, const void* x, const float* stats, const void* res, int relu, void* out, int M, int C,
                  hipStream_t stream) {
  MZ_CHECK_ARG(x && stats && out && M > 0 && C > 0 && C % 4 == 0, -1);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(grid_for((size_t)M * C / 4)), dim3(256), 0, stream, (const T*)x, stats,
                       (const T*)res, relu, (T*)out, M, C);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_bn_backward(int dtype, void* dy, const void* y, const void* x, const float* stats, int M, int C,
                     float* dgamma, float* dbeta, void* dx, void* ws, long long ws_bytes, hipStream_t stream) {
  MZ_CHECK_ARG(dy && x && stats && dgamma && dbeta && dx && ws && M > 0 && C > 0 && C % 4 == 0, -1);
  const int rpc = BN_RPC;
  const int nchunk = (M + rpc - 1) / rpc;
  MZ_CHECK_ARG((long long)nchunk * C * (long long)sizeof(float2) + 3LL * C * 4 <= ws_bytes, -2);
  float2* part = (float2*)ws;
  float* coef = (float*)((char*)ws + (size_t)nchunk * C * sizeof(float2));
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(bn_bwd_partial_kernel<T>, dim3((C + 63) / 64, nchunk), dim3(256), 0, stream, (T*)dy,
                       (const T*)y, (const T*)x, stats, M, C, rpc, part);
    hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(C), dim3(64), 0, stream, (const float2*)part, nchunk,
                       M, C, stats, dgamma, dbeta, coef);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(grid_for((size_t)M * C / 4)), dim3(256), 0, stream, (const T*)dy,
                       (const T*)x, stats, (const float*)coef, (T*)dx, M, C);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_conv_wpack(int dtype, const float* w, void* wt, int Cout, int taps, int Cin, int cin_used, int flip,
                    hipStream_t stream) {
  MZ_CHECK_ARG(w && wt && Cout > 0 && taps > 0 && Cin > 0 && cin_used > 0 && cin_used <= Cin, -1);
  const size_t n = flip ? (size_t)cin_used * taps * Cout : (size_t)Cout * taps * Cin;
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(conv_wt_kernel<T>, dim3(grid_for(n)), dim3(256), 0, stream, w, (T*)wt, Cout, taps, Cin,
                       cin_used, flip);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

static long long wgrad_splits(long long M, long long tiles) {
  long long nsplit = (512 + tiles - 1) / tiles;  // >= 2 workgroups per CU
  const long long maxs = (M + 255) / 256;        // >= 256 rows per split
  if (nsplit > maxs) nsplit = maxs;
  return nsplit < 1 ? 1 : nsplit;
}

int mzba_conv_pack_bf16(const float* w, void* out, int Cout, int taps, int Cin, int N, int Cc, int flip, int layout,
                        long long pad, hipStream_t stream) {
  MZ_CHECK_ARG(w && out && Cout > 0 && Cin > 0 && N > 0 && Cc > 0 && pad >= 0 && (layout == 1 || layout == 2), -1);
  MZ_CHECK_ARG(layout != 1 || (N % 32 == 0 && Cc % 32 == 0), -2);
  MZ_CHECK_ARG(layout != 2 || (taps == 9 && N % 16 == 0 && Cc % 32 == 0), -3);
  MZ_CHECK_ARG(flip ? (N <= Cin && Cc == Cout) : (N == Cout && Cc <= Cin), -4);
  const size_t n = (size_t)N * taps * Cc + (size_t)pad;
  hipLaunchKernelGGL(conv_pack_kernel, dim3(grid_for(n)), dim3(256), 0, stream, w, (bf16_t*)out, Cout, taps, Cin, N, Cc,
                     flip, layout, (size_t)pad);
  MZ_LAUNCH_CHECK();
  return 0;
}

// njobs packs, each the arguments of one mzba_conv_pack_bf16 call: w[j], out[j] (16-B aligned) and
// prm[8 j ..] = {Cout, taps, Cin, N, Cc, flip, layout, pad}; the same outputs as the njobs separate calls, in
// launches of PK_MAX jobs
int mzba_conv_pack_bf16_multi(const float* const* w, void* const* out, const int* prm, int njobs, hipStream_t stream) {
  MZ_CHECK_ARG(w && out && prm && njobs > 0, -1);
  for (int j0 = 0; j0 < njobs; j0 += PK_MAX) {
    PackJobs js{};
    const int nj = njobs - j0 < PK_MAX ? njobs - j0 : PK_MAX;
    for (int k = 0; k < nj; ++k) {
      const int* p = prm + 8 * (j0 + k);
      const int Cout = p[0], taps = p[1], Cin = p[2], N = p[3], Cc = p[4], flip = p[5], layout = p[6], pad = p[7];
      MZ_CHECK_ARG(w[j0 + k] && out[j0 + k] && ((uintptr_t)out[j0 + k] & 15) == 0 && Cout > 0 && Cin > 0 && N > 0 &&
                       Cc > 0 && pad >= 0 && pad % 8 == 0 && (layout == 1 || layout == 2), -1);
      MZ_CHECK_ARG(layout != 1 || (N % 32 == 0 && Cc % 32 == 0), -2);
      MZ_CHECK_ARG(layout != 2 || (taps == 9 && N % 16 == 0 && Cc % 32 == 0), -3);
      MZ_CHECK_ARG(flip ? (N <= Cin && Cc == Cout) : (N == Cout && Cc <= Cin), -4);
      MZ_CHECK_ARG((long long)N * taps * Cc + pad < (1LL << 31), -5);
      js.j[k] = PackJob{w[j0 + k], (bf16_t*)out[j0 + k], Cout, taps, Cin, N, Cc, flip, layout, pad};
    }
    hipLaunchKernelGGL(conv_pack_multi_kernel, dim3(64, nj), dim3(256), 0, stream, js);
    MZ_LAUNCH_CHECK();
  }
  return 0;
}

static thread_local int g_wgrad_img = 1;
// 1 (default): bf16 3x3 weight gradients on the whole-image kernel where it wins (see
// wgrad_img_eligible); 2: whole-image kernel for every supported shape; 0: per-tap kernel only
int mzba_conv_wgrad_set_variant(int v) {
  if (v < 0 || v > 2) return -1;
  g_wgrad_img = v;
  return 0;
}
// which whole-image kernel: 2 (default) pixel rows with 64-co wave tiles (conv_wgrad_px_kernel<1>), 1 pixel
// rows with 32-co wave tiles (conv_wgrad_px_kernel<0>, the same bits, 3-6 % slower per launch), 0 zero-bordered
// images (conv_wgrad_img_kernel, the round-5 form); 1 and 0 for A/B; 3 = form 2 with the k steps
// software-pipelined (conv_wgrad_px_kernel<2>, the same bits)
static thread_local int g_wgrad_form = 2;
int mzba_conv_wgrad_set_form(int v) {
  if (v < 0 || v > 3) return -1;
  g_wgrad_form = v;
  return 0;
}

long long mzba_conv_wgrad_ws_bytes(int B, int H, int W, int Cin, int Cout, int ks) {
  const long long M = (long long)B * H * W;
  const long long tiles = (long long)((Cout + 63) / 64) * ((Cin + 63) / 64) * ks * ks;
  long long n = wgrad_splits(M, tiles);
  WgPlan p;
  if (ks == 3 && Cin % 8 == 0 && Cout % 8 == 0 && wgrad_img_plan(B, 1, H, W, Cin, Cout, p) && p.nsplit > n) n = p.nsplit;
  WgPxPlan px;
  if (ks == 3 && Cin % 8 == 0 && Cout % 8 == 0 && wgrad_px_plan(B, 1, H, W, Cin, Cout, px) && px.nsplit > n) n = px.nsplit;
  return n * ((long long)Cout * ks * ks * Cin + Cout) * 4;
}

// a whole-image kernel for nseg segments of B envs (its plan may still refuse the shape)
static bool wgrad_img_eligible(int dtype, int nseg, int B, int H, int W, int Cin, int Cout, int ks) {
  // it wins where an image has many pixels per tap re-read (8x10: 138 vs 277 us, 16x20: 153 vs
  // 283 us at B = 512) and, at 4x5, once the K unrolled uses of a conv reduce in one launch
  // (per-tap kernel: 80 us per use; 5 x 512 at 256 -> 256: 188 vs 401 us, and 362 vs 464 us for
  // the dynamics ConvBlock's 264 input channels; tools/bench_wgrad_segs.py)
  if (dtype != 1 || ks != 3 || !g_wgrad_img || Cin % 8 || Cout % 8) return false;
  return H * W >= 64 || g_wgrad_img == 2 || nseg * B >= 2048;
}

static int wgrad_core(int dtype, const void* const* xs, const void* const* dys, int nseg, int B, int H, int W, int Cin,
                      int Cout, int ks, float* dw, float* db, void* ws, long long ws_bytes, hipStream_t stream) {
  MZ_CHECK_ARG(xs && dys && dw && ws && B > 0 && nseg >= 1 && nseg <= WG_MAXSEG && (ks == 1 || ks == 3) &&
               Cin % 4 == 0 && Cout % 4 == 0, -1);
  MZ_CHECK_ARG(dtype == 0 || (Cin % 8 == 0 && Cout % 8 == 0), -1);
  MZ_CHECK_ARG(dtype == 0 || dtype == 1, -9);
  for (int i = 0; i < nseg; ++i) MZ_CHECK_ARG(xs[i] && dys[i], -1);
  MZ_CHECK_ARG(mzba_conv_wgrad_ws_bytes(nseg * B, H, W, Cin, Cout, ks) <= ws_bytes, -2);
  WgPxPlan pxp;
  if (g_wgrad_form >= 1 && wgrad_img_eligible(dtype, nseg, B, H, W, Cin, Cout, ks) &&
      wgrad_px_plan(nseg * B, B, H, W, Cin, Cout, pxp)) {
    static bool attr = false;
    if (!attr) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_px_kernel<0>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)WI_LDS_MAX);
      if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_px_kernel<1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)WI_LDS_MAX);
      if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_px_kernel<2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)WI_LDS_MAX);
      if (e != hipSuccess) return (int)e;
      attr = true;
    }
    for (int i = 0; i < nseg; ++i) {
      pxp.a.xs[i] = (const bf16_t*)xs[i];
      pxp.a.dys[i] = (const bf16_t*)dys[i];
    }
    const size_t nwi = (size_t)Cout * 9 * Cin;
    float* ipart = (float*)ws;
    float* ibpart = db ? ipart + (size_t)pxp.nsplit * nwi : nullptr;
    if (g_wgrad_form == 3)
      hipLaunchKernelGGL(conv_wgrad_px_kernel<2>, dim3(pxp.a.tiles, pxp.nsplit), dim3(WI_NT), pxp.lds, stream, pxp.a,
                         ipart, ibpart);
    else if (g_wgrad_form == 2)
      hipLaunchKernelGGL(conv_wgrad_px_kernel<1>, dim3(pxp.a.tiles, pxp.nsplit), dim3(WI_NT), pxp.lds, stream, pxp.a,
                         ipart, ibpart);
    else
      hipLaunchKernelGGL(conv_wgrad_px_kernel<0>, dim3(pxp.a.tiles, pxp.nsplit), dim3(WI_NT), pxp.lds, stream, pxp.a,
                         ipart, ibpart);
    const size_t nbi = db ? (size_t)Cout : 0;
    hipLaunchKernelGGL(sum_partials2_kernel, dim3(grid_for(nwi + nbi)), dim3(256), 0, stream, (const float*)ipart,
                       (const float*)ibpart, pxp.nsplit, nwi, nbi, dw, db);
    MZ_LAUNCH_CHECK();
    return 0;
  }
  WgPlan ip;
  if (wgrad_img_eligible(dtype, nseg, B, H, W, Cin, Cout, ks) && wgrad_img_plan(nseg * B, B, H, W, Cin, Cout, ip)) {
    static bool attr = false;  // the 16x20 images need more than the default 64 KB of dynamic LDS
    if (!attr) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_img_kernel<false>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)WI_LDS_MAX);
      if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_img_kernel<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)WI_LDS_MAX);
      if (e != hipSuccess) return (int)e;
      attr = true;
    }
    ip.a.Bseg = B;
    for (int i = 0; i < nseg; ++i) {
      ip.a.xs[i] = (const bf16_t*)xs[i];
      ip.a.dys[i] = (const bf16_t*)dys[i];
    }
    const size_t nwi = (size_t)Cout * 9 * Cin;
    float* ipart = (float*)ws;
    float* ibpart = db ? ipart + (size_t)ip.nsplit * nwi : nullptr;
    const dim3 grid(((Cout + 63) / 64) * ((Cin + 63) / 64), ip.nsplit);
    if (ip.pf)
      hipLaunchKernelGGL(conv_wgrad_img_kernel<true>, grid, dim3(WI_NT), ip.lds, stream, ip.a, ipart, ibpart);
    else
      hipLaunchKernelGGL(conv_wgrad_img_kernel<false>, grid, dim3(WI_NT), ip.lds, stream, ip.a, ipart, ibpart);
    const size_t nbi = db ? (size_t)Cout : 0;
    hipLaunchKernelGGL(sum_partials2_kernel, dim3(grid_for(nwi + nbi)), dim3(256), 0, stream, (const float*)ipart,
                       (const float*)ibpart, ip.nsplit, nwi, nbi, dw, db);
    MZ_LAUNCH_CHECK();
    return 0;
  }
  // per-tap tile kernels, one launch pair per segment (accumulated into dw / db in segment order)
  const long long M = (long long)B * H * W;
  const long long tiles = (long long)((Cout + 63) / 64) * ((Cin + 63) / 64) * ks * ks;
  const long long nsplit = wgrad_splits(M, tiles);
  const int step = dtype ? WB_M : WG_ROWS;
  const int rps = (int)(((M + nsplit - 1) / nsplit + step - 1) / step * step);
  const size_t nw = (size_t)Cout * ks * ks * Cin;
  float* part = (float*)ws;
  float* bpart = db ? part + nsplit * nw : nullptr;
  for (int i = 0; i < nseg; ++i) {
    if (dtype == 1)
      hipLaunchKernelGGL(conv_wgrad_bf16_kernel, dim3((unsigned)tiles, (unsigned)nsplit), dim3(256), 0, stream,
                         (const bf16_t*)xs[i], (const bf16_t*)dys[i], B, H, W, Cin, Cout, ks, rps, part, bpart);
    else
      hipLaunchKernelGGL(conv_wgrad_kernel<float>, dim3((unsigned)tiles, (unsigned)nsplit), dim3(256), 0, stream,
                         (const float*)xs[i], (const float*)dys[i], B, H, W, Cin, Cout, ks, rps, part, bpart);
    const size_t nb = db ? (size_t)Cout : 0;
    hipLaunchKernelGGL(sum_partials2_kernel, dim3(grid_for(nw + nb)), dim3(256), 0, stream, (const float*)part,
                       (const float*)bpart, (int)nsplit, nw, nb, dw, db);
  }
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_conv_wgrad(int dtype, const void* x, const void* dy, int B, int H, int W, int Cin, int Cout, int ks,
                    float* dw, float* db, void* ws, long long ws_bytes, hipStream_t stream) {
  return wgrad_core(dtype, &x, &dy, 1, B, H, W, Cin, Cout, ks, dw, db, ws, ws_bytes, stream);
}

int mzba_conv_wgrad_segs(int dtype, const void* const* xs, const void* const* dys, int nseg, int B, int H, int W,
                         int Cin, int Cout, int ks, float* dw, float* db, void* ws, long long ws_bytes,
                         hipStream_t stream) {
  return wgrad_core(dtype, xs, dys, nseg, B, H, W, Cin, Cout, ks, dw, db, ws, ws_bytes, stream);
}

int mzba_avgpool2_backward(int dtype, const void* dy, void* dx, int B, int H, int W, int C, hipStream_t stream) {
  MZ_CHECK_ARG(dy && dx && B > 0 && H % 2 == 0 && W % 2 == 0, -1);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    if (C % 4 == 0 && (long long)B * H * W * C < (1LL << 31))
      hipLaunchKernelGGL(avgpool2_bwd4_kernel<T>, dim3(grid_for((size_t)B * H * W * C / 4)), dim3(256), 0, stream,
                         (const T*)dy, (T*)dx, B, H, W, C);
    else
      hipLaunchKernelGGL(avgpool2_bwd_kernel<T>, dim3(grid_for((size_t)B * H * W * C)), dim3(256), 0, stream,
                         (const T*)dy, (T*)dx, B, H, W, C);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_axpy(int dtype, void* y, const void* x, long long n, hipStream_t stream) {
  MZ_CHECK_ARG(y && x && n >= 0, -1);
  if (n == 0) return 0;
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(axpy_kernel<T>, dim3(grid_for((size_t)n)), dim3(256), 0, stream, (T*)y, (const T*)x, (size_t)n);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_scale_forward(int dtype, const void* h, void* out, float* minmax, int32_t* argminmax, int B, int HW, int C,
                       hipStream_t stream) {
  MZ_CHECK_ARG(h && out && minmax && argminmax && B > 0 && HW > 0 && C > 0, -1);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(scale_fwd_kernel<T>, dim3(B), dim3(256), 0, stream, (const T*)h, (T*)out, (float2*)minmax,
                       (int2*)argminmax, HW, C);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_scale_backward(int dtype, const void* dy, const void* h, const float* minmax, const int32_t* argminmax,
                        void* dh, int B, int n, int accumulate, hipStream_t stream) {
  MZ_CHECK_ARG(dy && h && minmax && argminmax && dh && B > 0 && n > 0, -1);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(scale_bwd_kernel<T>, dim3(B), dim3(256), 0, stream, (const T*)dy, (const T*)h,
                       (const float2*)minmax, (const int2*)argminmax, (T*)dh, n, accumulate);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_linear_forward(int dtype, const void* x, const float* w, const float* bias, float* out, int B, int K, int O,
                        hipStream_t stream) {
  MZ_CHECK_ARG(x && w && bias && out && B > 0 && K > 0 && O > 0 && O <= 16, -1);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(linear_fwd_kernel<T>, dim3(B), dim3(256), 0, stream, (const T*)x, w, bias, out, K, O);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

long long mzba_linear_ws_bytes(int B, int K, int O) {
  const int nsplit = B >= 64 ? 16 : 1;
  return (long long)nsplit * ((long long)O * K + O) * 4;
}

int mzba_linear_backward(int dtype, const void* x, const float* w, const float* dy, void* dx, int accumulate,
                         float* dw, float* db, int B, int K, int O, void* ws, long long ws_bytes, hipStream_t stream) {
  MZ_CHECK_ARG(x && w && dy && dw && db && ws && B > 0 && K > 0 && O > 0 && O <= 16, -1);
  MZ_CHECK_ARG(mzba_linear_ws_bytes(B, K, O) <= ws_bytes, -2);
  const int nsplit = B >= 64 ? 16 : 1;
  const int rps = (B + nsplit - 1) / nsplit;
  float* part = (float*)ws;
  float* bpart = part + (size_t)nsplit * O * K;
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    if (dx)
      hipLaunchKernelGGL(linear_bwd_x_kernel<T>, dim3(grid_for((size_t)B * K)), dim3(256), 0, stream, dy, w, (T*)dx, B,
                         K, O, accumulate);
    hipLaunchKernelGGL(linear_bwd_w_kernel<T>, dim3((K + 255) / 256, nsplit), dim3(256), 0, stream, dy, (const T*)x,
                       B, K, O, rps, part, bpart);
    hipLaunchKernelGGL(sum_partials2_kernel, dim3(grid_for((size_t)O * K + O)), dim3(256), 0, stream,
                       (const float*)part, (const float*)bpart, nsplit, (size_t)O * K, (size_t)O, dw, db);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_learner_loss(const float* logit_r, const float* logit_v, const float* logit_p, const float* rewards,
                      const float* targets, const float* counts, const int32_t* slots, int B, int K, int ns, int na,
                      float smin, float smax, float* dlogit_r, float* dlogit_v, float* dlogit_p, float* loss,
                      hipStream_t stream) {
  MZ_CHECK_ARG(logit_r && logit_v && logit_p && rewards && targets && counts && dlogit_r && dlogit_v && dlogit_p &&
                   loss && B > 0 && K > 0 && ns >= 2 && ns <= 16 && na > 0 && na <= 16,
               -1);
  hipLaunchKernelGGL(loss_kernel, dim3(1), dim3(LOSS_T), 0, stream, logit_r, logit_v, logit_p, rewards, targets, counts,
                     slots, B, K, ns, na, smin, smax, dlogit_r, dlogit_v, dlogit_p, loss);
  MZ_LAUNCH_CHECK();
  return 0;
}

long long mzba_learner_loss_ws_bytes(int B, int K) { return 3LL * B * K * (long long)sizeof(double); }

int mzba_learner_loss_ws(const float* logit_r, const float* logit_v, const float* logit_p, const float* rewards,
                         const float* targets, const float* counts, const int32_t* slots, int B, int K, int ns, int na,
                         float smin, float smax, float* dlogit_r, float* dlogit_v, float* dlogit_p, float* loss,
                         void* ws, long long ws_bytes, hipStream_t stream) {
  MZ_CHECK_ARG(logit_r && logit_v && logit_p && rewards && targets && counts && dlogit_r && dlogit_v && dlogit_p &&
                   loss && ws && B > 0 && K > 0 && ns >= 2 && ns <= 16 && na > 0 && na <= 16,
               -1);
  MZ_CHECK_ARG(mzba_learner_loss_ws_bytes(B, K) <= ws_bytes && (long long)B * K < (1LL << 28), -2);
  const int BK = B * K;
  hipLaunchKernelGGL(loss_rows_kernel, dim3((BK + 255) / 256), dim3(256), 0, stream, logit_r, logit_v, logit_p, rewards,
                     targets, counts, slots, B, K, ns, na, smin, smax, dlogit_r, dlogit_v, dlogit_p, (double*)ws);
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(LOSS_T), 0, stream, (const double*)ws, B, K, loss);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_adam(float* p, const float* grad, float* m, float* v, long long n, float neg_step, float one_m_b1, float b2,
              float one_m_b2, float bc2_sqrt, float eps, float weight_decay, hipStream_t stream) {
  MZ_CHECK_ARG(p && grad && m && v && n >= 0, -1);
  if (n == 0) return 0;
  const bool a16 = (((uintptr_t)p | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
  if (n % 4 == 0 && a16)
    hipLaunchKernelGGL(adam4_kernel<false>, dim3(grid_for((size_t)n / 4)), dim3(256), 0, stream, (float4*)p,
                       (const float4*)grad, (float4*)m, (float4*)v, (size_t)n / 4, nullptr, neg_step, one_m_b1, b2,
                       one_m_b2, bc2_sqrt, eps, weight_decay);
  else
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for((size_t)n)), dim3(256), 0, stream, p, grad, m, v, (size_t)n, neg_step,
                       one_m_b1, b2, one_m_b2, bc2_sqrt, eps, weight_decay);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_adam_dev(float* p, const float* grad, float* m, float* v, long long n, const float* scalars,
                  hipStream_t stream) {
  MZ_CHECK_ARG(p && grad && m && v && scalars && n >= 0, -1);
  if (n == 0) return 0;
  const bool a16 = (((uintptr_t)p | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
  if (n % 4 == 0 && a16)
    hipLaunchKernelGGL(adam4_kernel<true>, dim3(grid_for((size_t)n / 4)), dim3(256), 0, stream, (float4*)p,
                       (const float4*)grad, (float4*)m, (float4*)v, (size_t)n / 4, scalars, 0.f, 0.f, 0.f, 0.f, 0.f,
                       0.f, 0.f);
  else
    hipLaunchKernelGGL(adam_dev_kernel, dim3(grid_for((size_t)n)), dim3(256), 0, stream, p, grad, m, v, (size_t)n,
                       scalars);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_learner_input(int dtype, const uint8_t* states, const int64_t* past_actions, const int32_t* slots,
                       const float* lut8, void* out, int B, int L, int HW, int Cp, hipStream_t stream) {
  MZ_CHECK_ARG(states && past_actions && slots && lut8 && out && B > 0 && L > 0 && Cp >= 2 * L, -1);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(learner_input_kernel<T>, dim3(grid_for((size_t)B * HW * Cp)), dim3(256), 0, stream, states,
                       past_actions, slots, lut8, (T*)out, B, L, HW, Cp);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

int mzba_dyn_input(int dtype, const void* h, const int64_t* future_actions, const int32_t* slots, int K, int k,
                   void* out, int B, int HW, int C, int A, int Cp, hipStream_t stream) {
  MZ_CHECK_ARG(h && future_actions && slots && out && B > 0 && k >= 0 && k < K && Cp >= C + A, -1);
  return dispatch(dtype, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(dyn_input_kernel<T>, dim3(grid_for((size_t)B * HW * Cp)), dim3(256), 0, stream, (const T*)h,
                       future_actions, slots, K, k, (T*)out, B, HW, C, A, Cp);
    MZ_LAUNCH_CHECK();
    return 0;
  });
}

}  // extern "C"
