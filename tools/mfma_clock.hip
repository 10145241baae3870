// MFMA shape vs held clock: does v_mfma_f32_32x32x16_bf16 hold a higher clock, or a higher
// FLOP rate, than v_mfma_f32_16x16x32_bf16 under the same sustained all-CU load? Register-only MFMA streams (no
// memory in the loop), 2 waves per SIMD, NACC independent accumulator chains per wave, every CU busy for ~20 ms.
// Per workgroup, wave 0 records s_memtime (core clock) and s_memrealtime (100 MHz) around its loop, so each
// launch reports the achieved dense FLOP rate (HIP events) and the core clock the waves ran at. Wave 0 is the older
// wave of its SIMD and runs its MFMAs mostly ahead of its partner (oldest-first issue), so its stamps cover about
// the first half of the launch: its cycles per 32 K FLOP are the issue cost of one wave's stream while the other
// waits, and the clock is the clock of that half.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_clock.hip -o tools/mfma_clock && ./tools/mfma_clock
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

// SHAPE 0: 16x16x32 (16 K FLOP per MFMA), 1: 32x32x16 (32 K FLOP per MFMA). NACC chains, ITERS loop trips.
template <int SHAPE, int NACC>
__global__ __launch_bounds__(512, 2) void mfma_loop(float* out, unsigned long long* stamps, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (lane + i));
    b[i] = (__bf16)(0.002f * (lane - i));
  }
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  float s = 0.f;
  if (SHAPE == 0) {
    f32x4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc[j], 0, 0, 0);
    }
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][3];
  } else {
    f32x16 acc[NACC];
    for (int j = 0; j < NACC; ++j)
      for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
    }
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][15];
  }
  if (threadIdx.x == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    stamps[2 * blockIdx.x] = t1 - t0;  // vector stores (thread 0's VGPRs)
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int SHAPE, int NACC>
int run(const char* name, int iters, int reps, int nblk) {
  float* out;
  unsigned long long* st;
  CHECK(hipMalloc(&out, sizeof(float) * nblk * 512));
  CHECK(hipMalloc(&st, sizeof(unsigned long long) * 2 * nblk));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // FLOP per launch: 8 waves x iters x (SHAPE 0: 2 NACC MFMAs of 16 K; 1: NACC MFMAs of 32 K)
  const double fl = 8.0 * nblk * iters * NACC * 32768.0;
  hipLaunchKernelGGL((mfma_loop<SHAPE, NACC>), dim3(nblk), dim3(512), 0, 0, out, st, iters);  // warm-up
  CHECK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((mfma_loop<SHAPE, NACC>), dim3(nblk), dim3(512), 0, 0, out, st, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(2 * nblk);
    CHECK(hipMemcpy(h.data(), st, sizeof(unsigned long long) * 2 * nblk, hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int i = 0; i < nblk; ++i) {
      cyc += h[2 * i];
      real += h[2 * i + 1];
    }
    const double ghz = cyc / (real / 100e6) / 1e9;  // s_memrealtime runs at 100 MHz
    printf("{\"shape\": \"%s\", \"nacc\": %d, \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"frac_2500\": %.4f, "
           "\"core_ghz\": %.3f, \"wave0_cycles_per_32k_flop\": %.2f}\n",
           name, NACC, r, ms, fl / ms / 1e9, fl / ms / 1e9 / 2500.0, ghz,
           (cyc / nblk) / ((double)iters * NACC));
    fflush(stdout);
  }
  CHECK(hipFree(out));
  CHECK(hipFree(st));
  return 0;
}

int main() {
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int nblk = ncu;  // one 8-wave workgroup per CU (2 waves per SIMD)
  for (int pass = 0; pass < 2; ++pass) {  // alternated, so a drifting clock shows in both shapes
    if (run<0, 4>("16x16x32", 200000, 3, nblk)) return 1;
    if (run<1, 4>("32x32x16", 200000, 3, nblk)) return 1;
    if (run<0, 8>("16x16x32", 100000, 3, nblk)) return 1;
    if (run<1, 8>("32x32x16", 100000, 3, nblk)) return 1;
  }
  return 0;
}
