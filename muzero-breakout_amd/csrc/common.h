// Common device helpers for the MI355X (gfx950) MuZero-Breakout acting path.
// Compiled with -ffp-contract=off: every f32 expression below is evaluated op by
// op, matching the reference's chains of separate f32 torch ops.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/mzba.h"  // declarations checked against the definitions

#define MZ_DEV __device__ __forceinline__

// hipFuncAttributeMaxDynamicSharedMemorySize for a kernel, set once per kernel pointer (a launch helper
// shared by several template instances must not key the one-time flag on the helper: ADVICE r4)
#include <mutex>
#include <set>
inline void mz_set_lds_max_once(const void* kern, int bytes) {
  static std::mutex mu;
  static std::set<const void*> done;
  std::lock_guard<std::mutex> lk(mu);
  if (done.insert(kern).second) (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// ------------------------------------------------------------------ error plumbing
// Every C-ABI entry point returns 0 on success, a negative code on a bad argument,
// or the positive hipError_t of the failing launch.
#define MZ_CHECK_ARG(cond, code) \
  do {                           \
    if (!(cond)) return (code);  \
  } while (0)
#define MZ_LAUNCH_CHECK()                    \
  do {                                       \
    hipError_t e__ = hipGetLastError();      \
    if (e__ != hipSuccess) return (int)e__;  \
  } while (0)

// ------------------------------------------------------------------ bf16
typedef uint16_t bf16_t;
MZ_DEV float bf16_to_f32(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
typedef __attribute__((ext_vector_type(2))) __bf16 mz_bf16x2;
// round-to-nearest-even; gfx950 converts in hardware (v_cvt_pk_bf16_f32)
MZ_DEV bf16_t f32_to_bf16(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
MZ_DEV uint32_t pack_bf16x2(float lo, float hi) {
  const mz_bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

template <typename T> struct ElemIO;
template <> struct ElemIO<float> {
  static MZ_DEV float load(const float* p) { return *p; }
  static MZ_DEV void store(float* p, float v) { *p = v; }
};
template <> struct ElemIO<bf16_t> {
  static MZ_DEV float load(const bf16_t* p) { return bf16_to_f32(*p); }
  static MZ_DEV void store(bf16_t* p, float v) { *p = f32_to_bf16(v); }
};

// ------------------------------------------------------------------ Philox4x32-10
// Bit-identical to oracle/rng.py. Counter = (global env, stream, step, call).
enum { MZ_STREAM_RESET = 0, MZ_STREAM_TIE = 1, MZ_STREAM_NOISE = 2, MZ_STREAM_SAMPLE = 3 };

struct u32x4 { uint32_t x, y, z, w; };

MZ_DEV u32x4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return {c0, c1, c2, c3};
}
MZ_DEV uint32_t mz_u32(uint32_t env, uint32_t stream, uint32_t step, uint32_t call, uint64_t seed) {
  return philox4x32(env, stream, step, call, seed).x;
}
MZ_DEV float mz_uniform(uint32_t env, uint32_t stream, uint32_t step, uint32_t call, uint64_t seed) {
  return (float)(mz_u32(env, stream, step, call, seed) >> 8) * (1.0f / 16777216.0f);
}
MZ_DEV int mz_randbelow(uint32_t env, uint32_t stream, uint32_t step, uint32_t call, uint64_t seed, uint32_t n) {
  uint64_t x = mz_u32(env, stream, step, call, seed) >> 8;
  return (int)((x * (uint64_t)n) >> 24);
}

// ScalarTransforms.inverted_softmax_expectation (utils.py:74-81) for n <= 16 logits: softmax,
// expectation over torch.linspace(smin, smax, n), then the reference's inverse transform.
MZ_DEV float decode_support(const float* l, int n, float smin, float smax) {
  float m = l[0];
  for (int i = 1; i < n; ++i) m = fmaxf(m, l[i]);
  float e[16];
  float s = 0.f;
  for (int i = 0; i < n; ++i) { e[i] = expf(l[i] - m); s = s + e[i]; }
  const float step = (smax - smin) / (float)(n - 1);
  float x = 0.f;
  for (int i = 0; i < n; ++i) {
    float sup = smin + (float)i * step;  // torch.linspace(smin, smax, n)
    x = x + (e[i] / s) * sup;
  }
  float t = fabsf(x) + 0.999f;  // utils.py:28, epsilon 0.001
  float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
  return sg * (t * t - 1.f);
}
