// Linear heads + decode (networks.py:138-149, 200-223; utils.py:74-81; mcts.py:97-100,
// 197-199). Up to two heads per launch, one workgroup per env:
//   logits_h = X_h[b] (flattened NHWC, K_h) . W_h^T + b_h   (W_h permuted on the host from
//   torch's (c,h,w) flatten order to this (h,w,c) order), then
//   decode_h = 0: softmax over the outputs (policy)            -> dec[b][o]
//   decode_h = 1: support expectation + inverse transform       -> dec[b]
#include "common.h"

namespace {

constexpr int MAXO = 16;

struct HeadArgs {
  const void* x[2];
  const float* w[2];
  const float* bias[2];
  float* logits[2];  // optional [B][O]
  float* dec[2];     // [B][O] (softmax) or [B] (value)
  int K[2], O[2], decode[2];
  int nheads;
  float smin, smax;
};

// EPB envs per workgroup (round 5: one env per workgroup re-read the whole weight matrix — 225 KB for the reward
// head's 5120 x 11 — per env, 0.9 GB of L2 reads per launch at B = 4096; now once per EPB envs). Per env the sum
// order is unchanged: thread tid accumulates k = tid, tid + 256, ... in sequence, then the wave's xor-shuffle
// tree, then ((w0 + w1) + (w2 + w3)) + bias: the outputs are bit-identical to the one-env form.
template <typename T, int EPB>
__global__ __launch_bounds__(256) void heads_kernel(HeadArgs a, int B) {
  const int b0 = blockIdx.x * EPB, tid = threadIdx.x;
  __shared__ float red[4][EPB][2][MAXO];
  for (int h = 0; h < a.nheads; ++h) {
    const int K = a.K[h], O = a.O[h];
    const float* w = a.w[h];
    const T* x[EPB];
#pragma unroll
    for (int e = 0; e < EPB; ++e) x[e] = (const T*)a.x[h] + (size_t)min(b0 + e, B - 1) * K;
    float acc[EPB][MAXO];
#pragma unroll
    for (int e = 0; e < EPB; ++e)
#pragma unroll
      for (int o = 0; o < MAXO; ++o) acc[e][o] = 0.f;
    // four k iterations' loads in flight (a rolled loop waited one memory round trip per iteration); per env and
    // output the adds stay in k order
#pragma unroll 4
    for (int k = tid; k < K; k += 256) {
      float xv[EPB];
#pragma unroll
      for (int e = 0; e < EPB; ++e) xv[e] = ElemIO<T>::load(x[e] + k);
#pragma unroll
      for (int o = 0; o < MAXO; ++o)
        if (o < O) {
          const float wv = w[(size_t)o * K + k];
#pragma unroll
          for (int e = 0; e < EPB; ++e) acc[e][o] = acc[e][o] + xv[e] * wv;
        }
    }
#pragma unroll
    for (int e = 0; e < EPB; ++e)
#pragma unroll
      for (int o = 0; o < MAXO; ++o) {
        float v = acc[e][o];
        for (int s = 32; s > 0; s >>= 1) v = v + __shfl_xor(v, s);
        if ((tid & 63) == 0) red[tid >> 6][e][h][o] = v;
      }
  }
  __syncthreads();
  if (tid < EPB * a.nheads) {
    const int e = tid % EPB, h = tid / EPB, b = b0 + e;
    if (b >= B) return;
    float l[MAXO];
    for (int o = 0; o < a.O[h]; ++o) {
      l[o] = ((red[0][e][h][o] + red[1][e][h][o]) + (red[2][e][h][o] + red[3][e][h][o])) + a.bias[h][o];
      if (a.logits[h]) a.logits[h][(size_t)b * a.O[h] + o] = l[o];
    }
    if (a.decode[h] == 0) {
      float m = l[0];
      for (int o = 1; o < a.O[h]; ++o) m = fmaxf(m, l[o]);
      float ex[MAXO], sum = 0.f;
      for (int o = 0; o < a.O[h]; ++o) { ex[o] = expf(l[o] - m); sum = sum + ex[o]; }
      for (int o = 0; o < a.O[h]; ++o) a.dec[h][(size_t)b * a.O[h] + o] = ex[o] / sum;
    } else {
      a.dec[h][b] = decode_support(l, a.O[h], a.smin, a.smax);
    }
  }
}

// bf16 path: the heads as a small MFMA GEMM. A workgroup = 16 envs x 16 (padded) outputs;
// 8 waves split K; v_mfma_f32_16x16x32_bf16 with A = activations (lane: env l&15, 8 k),
// B = bf16 weights Wb[16][K] (lane: output l&15, 8 k); partial sums reduced through LDS.
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct HeadArgsB {
  const bf16_t* x[2];
  const bf16_t* w[2];  // [16][K] (rows >= O are zero)
  const float* bias[2];
  float* logits[2];
  float* dec[2];
  int K[2], O[2], decode[2];
  int nheads, B;
  float smin, smax;
};

__global__ __launch_bounds__(512) void heads_mfma_kernel(HeadArgsB a) {
  __shared__ float part[8][16][17];
  __shared__ float lg[2][16][MAXO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int e0 = blockIdx.x * 16;
  const int el = lane & 15, q = lane >> 4;
  for (int hd = 0; hd < a.nheads; ++hd) {
    const int K = a.K[hd];
    const int env = min(e0 + el, a.B - 1);
    const bf16_t* xr = a.x[hd] + (size_t)env * K;
    const bf16_t* wr = a.w[hd] + (size_t)el * K;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int nk = K / 32;
    for (int s = wave; s < nk; s += 8) {
      const int k = s * 32 + q * 8;
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(xr + k);
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(wr + k);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
    }
    // D[row = env 4q + i][col = output el]
#pragma unroll
    for (int i = 0; i < 4; ++i) part[wave][4 * q + i][el] = acc[i];
    __syncthreads();
    if (tid < 256) {
      const int e = tid >> 4, o = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v = v + part[w][e][o];
      if (o < a.O[hd]) lg[hd][e][o] = v + a.bias[hd][o];
    }
    __syncthreads();
  }
  if (tid < 16 * a.nheads) {
    const int hd = tid >> 4, e = tid & 15, b = e0 + e;
    if (b < a.B) {
      const int O = a.O[hd];
      float l[MAXO];
      for (int o = 0; o < O; ++o) {
        l[o] = lg[hd][e][o];
        if (a.logits[hd]) a.logits[hd][(size_t)b * O + o] = l[o];
      }
      if (a.decode[hd] == 0) {
        float m = l[0];
        for (int o = 1; o < O; ++o) m = fmaxf(m, l[o]);
        float ex[MAXO], s = 0.f;
        for (int o = 0; o < O; ++o) { ex[o] = expf(l[o] - m); s = s + ex[o]; }
        for (int o = 0; o < O; ++o) a.dec[hd][(size_t)b * O + o] = ex[o] / s;
      } else {
        a.dec[hd][b] = decode_support(l, O, a.smin, a.smax);
      }
    }
  }
}

// f32 path (round 5): the heads as an f32 MFMA GEMM (v_mfma_f32_16x16x4_f32, the f32 convs' arithmetic: f32
// products accumulated in f32), 16 envs x 16 (padded) outputs per workgroup, 8 waves splitting K. A lane loads
// 4 consecutive k (16 B) of its env row and of its output's weight row; MFMA i of a 16-k step sums k = 16 s + 4 q + i
// over the four lane quarters q. The one-env-per-workgroup FMA form (heads_kernel) spent its time in 128 xor-shuffle
// reduction chains per launch (123 us at B = 4096 vs ~20 us of HBM reads).
__global__ __launch_bounds__(512) void heads_mfma_f32_kernel(HeadArgs a, int B) {
  __shared__ float part[8][16][17];
  __shared__ float lg[2][16][MAXO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int e0 = blockIdx.x * 16;
  const int el = lane & 15, q = lane >> 4;
  for (int hd = 0; hd < a.nheads; ++hd) {
    const int K = a.K[hd], O = a.O[hd];
    const int env = min(e0 + el, B - 1);
    const float* xr = (const float*)a.x[hd] + (size_t)env * K;
    const float* wr = a.w[hd] + (size_t)min(el, O - 1) * K;
    const bool wok = el < O;
    // four accumulators (one per 4-k component): each sums a quarter of the wave's products, then pairwise
    f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int ns = K / 16;
    for (int s = wave; s < ns; s += 8) {
      const int k = s * 16 + q * 4;
      const float4 xv = *reinterpret_cast<const float4*>(xr + k);
      float4 wv = *reinterpret_cast<const float4*>(wr + k);
      if (!wok) wv = make_float4(0.f, 0.f, 0.f, 0.f);
      // D[row = env][col = output]: A = activations (row el), B = weights (col el)
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.x, wv.x, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.y, wv.y, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.z, wv.z, acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.w, wv.w, acc[3], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) part[wave][4 * q + i][el] = (acc[0][i] + acc[1][i]) + (acc[2][i] + acc[3][i]);
    __syncthreads();
    if (tid < 256) {
      const int e = tid >> 4, o = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; w += 2) v = v + (part[w][e][o] + part[w + 1][e][o]);
      if (o < O) lg[hd][e][o] = v + a.bias[hd][o];
    }
    __syncthreads();
  }
  if (tid < 16 * a.nheads) {
    const int hd = tid >> 4, e = tid & 15, b = e0 + e;
    if (b < B) {
      const int O = a.O[hd];
      float l[MAXO];
      for (int o = 0; o < O; ++o) {
        l[o] = lg[hd][e][o];
        if (a.logits[hd]) a.logits[hd][(size_t)b * O + o] = l[o];
      }
      if (a.decode[hd] == 0) {
        float m = l[0];
        for (int o = 1; o < O; ++o) m = fmaxf(m, l[o]);
        float ex[MAXO], sm = 0.f;
        for (int o = 0; o < O; ++o) { ex[o] = expf(l[o] - m); sm = sm + ex[o]; }
        for (int o = 0; o < O; ++o) a.dec[hd][(size_t)b * O + o] = ex[o] / sm;
      } else {
        a.dec[hd][b] = decode_support(l, O, a.smin, a.smax);
      }
    }
  }
}

// ScalarTransforms.inverted_softmax_expectation over rows of n logits (utils.py:74-81)
__global__ void support_decode_kernel(const float* __restrict__ logits, float* __restrict__ out, int rows, int n,
                                      float smin, float smax) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float l[MAXO];
  for (int i = 0; i < n; ++i) l[i] = logits[(size_t)r * n + i];
  out[r] = decode_support(l, n, smin, smax);
}

}  // namespace

static int g_heads_mfma = 1;  // f32 heads: 1 the MFMA form (default), 0 the FMA form (heads_kernel; A/B, tests)

extern "C" {

int mzba_heads_set_variant(int v) {
  if (v != 0 && v != 1) return -1;
  g_heads_mfma = v;
  return 0;
}

int mzba_support_decode(const float* logits, float* out, int rows, int n, float smin, float smax,
                        hipStream_t stream) {
  MZ_CHECK_ARG(rows > 0 && n > 1 && n <= MAXO, -1);
  hipLaunchKernelGGL(support_decode_kernel, dim3((rows + 255) / 256), dim3(256), 0, stream, logits, out, rows, n, smin,
                     smax);
  MZ_LAUNCH_CHECK();
  return 0;
}


// bf16 MFMA heads: x*: [B][K] bf16, w*: [16][K] bf16 (zero rows >= O), K % 32 == 0.
int mzba_heads_bf16(int nheads, const void* x0, const void* w0, const float* b0, int K0, int O0, int dec0,
                    float* logits0, float* out0, const void* x1, const void* w1, const float* b1, int K1, int O1,
                    int dec1, float* logits1, float* out1, float smin, float smax, int B, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nheads >= 1 && nheads <= 2 && O0 > 0 && O0 <= MAXO && K0 % 32 == 0, -1);
  MZ_CHECK_ARG(nheads == 1 || (O1 > 0 && O1 <= MAXO && K1 % 32 == 0), -1);
  HeadArgsB a{{(const bf16_t*)x0, (const bf16_t*)x1}, {(const bf16_t*)w0, (const bf16_t*)w1}, {b0, b1},
              {logits0, logits1}, {out0, out1}, {K0, K1}, {O0, O1}, {dec0, dec1}, nheads, B, smin, smax};
  hipLaunchKernelGGL(heads_mfma_kernel, dim3((B + 15) / 16), dim3(512), 0, stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}


static inline bool a16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// x*: [B][K] activations (dtype 0 f32 / 1 bf16); w*: [O][K] f32; decode 0 softmax, 1 support
int mzba_heads(int dtype, int nheads, const void* x0, const float* w0, const float* b0, int K0, int O0, int dec0,
               float* logits0, float* out0, const void* x1, const float* w1, const float* b1, int K1, int O1,
               int dec1, float* logits1, float* out1, float smin, float smax, int B, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nheads >= 1 && nheads <= 2 && O0 <= MAXO && O0 > 0, -1);
  MZ_CHECK_ARG(nheads == 1 || (O1 <= MAXO && O1 > 0), -1);
  HeadArgs a{{x0, x1}, {w0, w1}, {b0, b1}, {logits0, logits1}, {out0, out1}, {K0, K1}, {O0, O1}, {dec0, dec1},
             nheads, smin, smax};
  constexpr int EPB = 8;
  const dim3 grid((unsigned)((B + EPB - 1) / EPB));
  if (dtype)
    hipLaunchKernelGGL((heads_kernel<bf16_t, EPB>), grid, dim3(256), 0, stream, a, B);
  else if (g_heads_mfma && K0 % 16 == 0 && (nheads == 1 || K1 % 16 == 0) && a16(x0) && a16(w0) &&
           (nheads == 1 || (a16(x1) && a16(w1))))  // its float4 loads: 16-B aligned bases (else the scalar form)
    hipLaunchKernelGGL(heads_mfma_f32_kernel, dim3((B + 15) / 16), dim3(512), 0, stream, a, B);
  else
    hipLaunchKernelGGL((heads_kernel<float, EPB>), grid, dim3(256), 0, stream, a, B);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
