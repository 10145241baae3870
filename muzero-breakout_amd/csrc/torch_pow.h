// Device restatement of the reference's temperature power `visit_counts ** (1/self.temperature)`
// (train_torch.py:192, and :574 in run_test_simulation) as torch 2.10 evaluates it on the CPU:
// the int64 counts become f32, then aten/native/cpu/PowKernel.cpp `pow_tensor_scalar_kernel`:
//   e == 0 -> 1; e == 1 -> copy; e == 0.5 -> sqrt; e == 2 -> b*b; e == 3 -> b*b*b;
//   otherwise `cpu_kernel_vec`: the flat elements [0, n - n % VB) of the (B, 3) batch tensor take the
//   vector lambda, SLEEF `Sleef_powf16_u10(b, f32(e))` (AVX512 host: VB = 32 floats per unrolled
//   iteration), the last n % VB take the scalar lambda `std::pow(float b, double e)` = f32(pow(double)).
// SLEEF's published powf_u10 (xpowf = expkf(dfmul(logkf(x), y)), double-float arithmetic with FMA)
// is restated for finite x >= 0, y > 0 — the only inputs visit counts produce. Needs exact f32
// division, fmaf and the op order below: compiled with -ffp-contract=off. Pinned bit for bit against
// torch (tests/golden/sampling.npz; oracle/torch_pow.c is the CPU twin used by the tests).
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>

namespace mzpow {

struct F2 {
  float x, y;
};
__device__ __forceinline__ F2 mk(float x, float y) { return F2{x, y}; }
__device__ __forceinline__ F2 normalize(F2 t) {
  const float s = t.x + t.y;
  return mk(s, (t.x - s) + t.y);
}
__device__ __forceinline__ F2 add_f2f2(F2 x, F2 y) {
  const float s = x.x + y.x;
  return mk(s, (((x.x - s) + y.x) + x.y) + y.y);
}
__device__ __forceinline__ F2 add_ff2(float x, F2 y) {
  const float s = x + y.x;
  return mk(s, ((x - s) + y.x) + y.y);
}
__device__ __forceinline__ F2 add2_ff(float x, float y) {
  const float s = x + y, v = s - x;
  return mk(s, (x - (s - v)) + (y - v));
}
__device__ __forceinline__ F2 add2_f2f(F2 x, float y) {
  const float s = x.x + y, v = s - x.x;
  return mk(s, ((x.x - (s - v)) + (y - v)) + x.y);
}
__device__ __forceinline__ F2 add2_f2f2(F2 x, F2 y) {
  const float s = x.x + y.x, v = s - x.x;
  return mk(s, ((x.x - (s - v)) + (y.x - v)) + (x.y + y.y));
}
__device__ __forceinline__ F2 scale(F2 d, float s) { return mk(d.x * s, d.y * s); }
__device__ __forceinline__ F2 sqr(F2 x) {
  const float s = x.x * x.x;
  return mk(s, __builtin_fmaf(x.x + x.x, x.y, __builtin_fmaf(x.x, x.x, -s)));
}
__device__ __forceinline__ F2 mul_f2f2(F2 x, F2 y) {
  const float s = x.x * y.x;
  return mk(s, __builtin_fmaf(x.x, y.y, __builtin_fmaf(x.y, y.x, __builtin_fmaf(x.x, y.x, -s))));
}
__device__ __forceinline__ F2 mul_f2f(F2 x, float y) {
  const float s = x.x * y;
  return mk(s, __builtin_fmaf(x.y, y, __builtin_fmaf(x.x, y, -s)));
}
__device__ __forceinline__ F2 div(F2 n, F2 d) {
  const float t = 1.0f / d.x, s = n.x * t;
  const float u = __builtin_fmaf(t, n.x, -s);
  const float v = __builtin_fmaf(-d.y, t, __builtin_fmaf(-d.x, t, 1.0f));
  return mk(s, __builtin_fmaf(s, v, __builtin_fmaf(n.y, t, u)));
}

// log(d) as a double-float for finite d > 0: d = m * 2^e, m in [0.75, 1.5)
__device__ __forceinline__ F2 logk(float d) {
  int e;
  frexpf(d * (1.0f / 0.75f), &e);
  e -= 1;
  const float m = ldexpf(d, -e);
  F2 s = mul_f2f(mk(0.69314718246459960938f, -1.904654323148236017e-09f), (float)e);
  const F2 x = div(add2_ff(-1.0f, m), add2_ff(1.0f, m));
  const F2 x2 = sqr(x);
  float t = 0.240320354700088500976562f;
  t = __builtin_fmaf(t, x2.x, 0.285112679004669189453125f);
  t = __builtin_fmaf(t, x2.x, 0.400007992982864379882812f);
  const F2 c = mk(0.66666662693023681640625f, 3.69183861259614332084311e-09f);
  s = add_f2f2(s, scale(x, 2.0f));
  return add_f2f2(s, mul_f2f2(mul_f2f2(x2, x), add2_f2f2(mul_f2f(x2, t), c)));
}

__device__ __forceinline__ float expk(F2 d) {
  float u = (d.x + d.y) * 1.442695040888963407359924681001892137426645954152985934135449406931f;
  const int q = (int)rintf(u);
  F2 s = add2_f2f(d, (float)q * -0.693145751953125f);
  s = add2_f2f(s, (float)q * -1.428606765330187045e-06f);
  s = normalize(s);
  u = 0.00136324646882712841033936f;
  u = __builtin_fmaf(u, s.x, 0.00836596917361021041870117f);
  u = __builtin_fmaf(u, s.x, 0.0416710823774337768554688f);
  u = __builtin_fmaf(u, s.x, 0.166665524244308471679688f);
  u = __builtin_fmaf(u, s.x, 0.499999850988388061523438f);
  F2 t = add_f2f2(s, mul_f2f(sqr(s), u));
  t = add_ff2(1.0f, t);
  u = ldexpf(t.x + t.y, q);
  return d.x < -104.0f ? 0.0f : u;
}

// Sleef_powf_u10(x, y) for finite x >= 0, y > 0
__device__ __forceinline__ float sleef_powf_u10(float x, float y) {
  if (x == 1.0f) return 1.0f;
  if (x == 0.0f) return 0.0f;
  return expk(mul_f2f(logk(x), y));
}

// The SIMD / scalar lane of the element at flat position idx of a tensor of n_total elements: torch's
// TensorIterator::for_each splits tensors of >= 32768 elements over its intra-op threads (at::parallel_for
// chunks of `chunk` elements; chunk = n_total when serial) and each chunk runs the vectorized loop over
// its first len - len % vb elements, the rest (its tail) through the scalar op
__device__ __forceinline__ bool torch_vec_lane(long long idx, long long chunk, long long n_total, int vb) {
  const long long c0 = idx / chunk * chunk;
  const long long len = (c0 + chunk < n_total ? c0 + chunk : n_total) - c0;
  return idx - c0 < len - len % vb;
}

// one element of torch's CPU `int64 counts ** e` at flat position `idx` of the batch tensor
__device__ __forceinline__ float torch_cpu_pow(long long count, double e, long long idx, long long chunk,
                                               long long n_total, int vb) {
  const float b = (float)count;
  if (e == 0.0) return 1.0f;
  if (e == 1.0) return b;
  if (e == 0.5) return sqrtf(b);
  if (e == 2.0) return b * b;
  if (e == 3.0) return b * b * b;
  if (torch_vec_lane(idx, chunk, n_total, vb)) return sleef_powf_u10(b, (float)e);
  return (float)pow((double)b, e);
}

// elements per intra-op thread chunk for a tensor of n_total elements evaluated with `threads` threads
// (at::internal::GRAIN_SIZE = 32768: serial below it; else min(threads, ceil(n / grain)) chunks)
inline long long torch_pow_chunk(long long n_total, int threads) {
  constexpr long long GRAIN = 32768;
  if (threads <= 1 || n_total < GRAIN) return n_total;
  const long long num = std::min<long long>(threads, (n_total + GRAIN - 1) / GRAIN);
  return (n_total + num - 1) / num;
}

}  // namespace mzpow
