/* ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product path.
 *
 * Bit-level restatement of what `visit_counts ** (1/self.temperature)` (train_torch.py:192) computes on
 * the reference's CPU: torch 2.10 `pow(Tensor int64, Scalar double)` -> the int64 counts are first
 * converted to float32 (the common dtype), then aten/src/ATen/native/cpu/PowKernel.cpp
 * `pow_tensor_scalar_kernel` runs:
 *   exponent == 0 -> 1;  == 1 -> copy;  == 0.5 -> sqrt;  == 2 -> b*b;  == 3 -> b*b*b;
 *   otherwise `cpu_kernel_vec`: elements [0, n - n % VB) go through the vector lambda
 *   `Vectorized<float>::pow(float(e))` = SLEEF `Sleef_powf16_u10` (AVX512 host, VB = 32 floats per
 *   unrolled iteration; AVX2: Sleef_powf8_u10, VB = 16), the last n % VB elements through the scalar
 *   lambda `std::pow(float b, double e)` = f32(pow(double b, e)) (glibc).
 * SLEEF is a third-party dependency of torch (vendored inside libtorch_cpu, pinned by torch 2.10.0);
 * its published powf_u10 algorithm (xpowf = expkf(dfmul(logkf(|x|), y)) in double-float arithmetic
 * with FMA) is restated below for finite x >= 0, y > 0 — the only inputs visit counts produce.
 * Pinned exhaustively against torch in this container: counts 0..1023 x every exponent of the
 * reference's temperature schedule, and 200 000 random (count, exponent) pairs, 0 mismatches
 * (tests/golden/sampling.npz, tests/test_oracle.py::test_torch_pow_oracle_matches_fixture).
 *
 * Build: gcc -O2 -ffp-contract=off -shared -fPIC oracle/torch_pow.c -lm (oracle/torch_pow.py does it).
 */
#include <math.h>
#include <stdint.h>

typedef struct { float x, y; } f2;
static f2 mk(float x, float y) { f2 r = {x, y}; return r; }
static f2 df_normalize(f2 t) { float s = t.x + t.y; return mk(s, (t.x - s) + t.y); }
static f2 df_add_f2f2(f2 x, f2 y) { float s = x.x + y.x; return mk(s, (((x.x - s) + y.x) + x.y) + y.y); }
static f2 df_add_ff2(float x, f2 y) { float s = x + y.x; return mk(s, ((x - s) + y.x) + y.y); }
static f2 df_add2_ff(float x, float y) {
  float s = x + y, v = s - x;
  return mk(s, (x - (s - v)) + (y - v));
}
static f2 df_add2_f2f(f2 x, float y) {
  float s = x.x + y, v = s - x.x;
  return mk(s, ((x.x - (s - v)) + (y - v)) + x.y);
}
static f2 df_add2_f2f2(f2 x, f2 y) {
  float s = x.x + y.x, v = s - x.x;
  return mk(s, ((x.x - (s - v)) + (y.x - v)) + (x.y + y.y));
}
static f2 df_scale(f2 d, float s) { return mk(d.x * s, d.y * s); }
static f2 df_sqr(f2 x) { float s = x.x * x.x; return mk(s, fmaf(x.x + x.x, x.y, fmaf(x.x, x.x, -s))); }
static f2 df_mul_f2f2(f2 x, f2 y) {
  float s = x.x * y.x;
  return mk(s, fmaf(x.x, y.y, fmaf(x.y, y.x, fmaf(x.x, y.x, -s))));
}
static f2 df_mul_f2f(f2 x, float y) { float s = x.x * y; return mk(s, fmaf(x.y, y, fmaf(x.x, y, -s))); }
static f2 df_div(f2 n, f2 d) {
  float t = 1.0f / d.x, s = n.x * t;
  float u = fmaf(t, n.x, -s);
  float v = fmaf(-d.y, t, fmaf(-d.x, t, 1.0f));
  return mk(s, fmaf(s, v, fmaf(n.y, t, u)));
}

/* log(d) as a double-float, d > 0 finite: d = m * 2^e with m in [0.75, 1.5) */
static f2 logk(float d) {
  int e;
  frexpf(d * (1.0f / 0.75f), &e);
  e -= 1;
  const float m = ldexpf(d, -e);
  f2 s = df_mul_f2f(mk(0.69314718246459960938f, -1.904654323148236017e-09f), (float)e);
  const f2 x = df_div(df_add2_ff(-1.0f, m), df_add2_ff(1.0f, m));
  const f2 x2 = df_sqr(x);
  float t = 0.240320354700088500976562f;
  t = fmaf(t, x2.x, 0.285112679004669189453125f);
  t = fmaf(t, x2.x, 0.400007992982864379882812f);
  const f2 c = mk(0.66666662693023681640625f, 3.69183861259614332084311e-09f);
  s = df_add_f2f2(s, df_scale(x, 2.0f));
  return df_add_f2f2(s, df_mul_f2f2(df_mul_f2f2(x2, x), df_add2_f2f2(df_mul_f2f(x2, t), c)));
}

static float expk(f2 d) {
  float u = (d.x + d.y) * 1.442695040888963407359924681001892137426645954152985934135449406931f;
  const int q = (int)rintf(u);
  f2 s = df_add2_f2f(d, (float)q * -0.693145751953125f);
  s = df_add2_f2f(s, (float)q * -1.428606765330187045e-06f);
  s = df_normalize(s);
  u = 0.00136324646882712841033936f;
  u = fmaf(u, s.x, 0.00836596917361021041870117f);
  u = fmaf(u, s.x, 0.0416710823774337768554688f);
  u = fmaf(u, s.x, 0.166665524244308471679688f);
  u = fmaf(u, s.x, 0.499999850988388061523438f);
  f2 t = df_add_f2f2(s, df_mul_f2f(df_sqr(s), u));
  t = df_add_ff2(1.0f, t);
  u = ldexpf(t.x + t.y, q);
  return d.x < -104.0f ? 0.0f : u;
}

/* Sleef_powf_u10 for x >= 0 finite, y > 0 finite */
float mz_sleef_powf_u10(float x, float y) {
  if (x == 1.0f) return 1.0f;
  if (x == 0.0f) return 0.0f;
  return expk(df_mul_f2f(logk(x), y));
}

/* torch CPU `int64 (B,3) ** e` (see header) for n elements that sit at flat positions
 * [start, start + n) of the reference's whole batch tensor of n_total = 3B elements (a shard of the
 * envs: start = 3 * env_offset); vb = 32 (AVX512 host) or 16 (AVX2). TensorIterator::for_each splits
 * tensors of >= 32768 elements over the intra-op threads (at::parallel_for: chunks of `chunk`
 * elements, oracle/torch_pow.py pow_chunk) and each chunk runs the vectorized loop with its own
 * scalar tail: element i takes the vector lane iff its offset in its chunk is below len - len % vb. */
void mz_torch_pow_counts(const int64_t* counts, float* out, long long n, double e, int vb, long long start,
                         long long n_total, long long chunk) {
  if (chunk <= 0) chunk = n_total;
  for (long long i = 0; i < n; ++i) {
    const float b = (float)counts[i];
    const long long g = start + i, c0 = g / chunk * chunk;
    const long long len = (c0 + chunk < n_total ? c0 + chunk : n_total) - c0;
    float r;
    if (e == 0.0) r = 1.0f;
    else if (e == 1.0) r = b;
    else if (e == 0.5) r = sqrtf(b);
    else if (e == 2.0) r = b * b;
    else if (e == 3.0) r = b * b * b;
    else if (g - c0 < len - len % vb) r = mz_sleef_powf_u10(b, (float)e);
    else r = (float)pow((double)b, e);
    out[i] = r;
  }
}
