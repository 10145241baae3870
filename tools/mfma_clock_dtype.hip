// Element type vs held clock: does v_mfma_f32_16x16x32_f16 hold a lower clock than
// v_mfma_f32_16x16x32_bf16 under the same sustained all-CU load? Config 5's fp16 dynamics step (towerp_kernel<1>)
// ran at 2.00 GHz against 2.085 GHz for the bf16 steps with the same instruction stream apart from the element type.
// Register-only MFMA streams (no memory, no VALU in the loop), 2 waves per SIMD, 4 independent accumulator chains per
// wave, operands from a per-lane hash of full-range values in the tower's magnitude (|x| ~ 0.01 - 4, random signs)
// rotated over 4 register pairs so consecutive MFMAs see different bits (constant operands would not toggle the
// multipliers). Per workgroup, wave 0 records s_memtime / s_memrealtime around its loop: the core clock it ran at.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_clock_dtype.hip -o tools/mfma_clock_dtype && ./tools/mfma_clock_dtype
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__device__ float hval(unsigned x) {  // a value in +-[0.01, 4) from a hash
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  const float m = 0.01f + 3.99f * (float)(x & 0xffff) / 65536.f;
  return (x & 0x10000) ? -m : m;
}

// EL 0 bf16, 1 fp16
template <int EL>
__global__ __launch_bounds__(512, 2) void mfma_loop(float* out, unsigned long long* stamps, int iters) {
  using V8 = typename std::conditional<EL == 0, bf16x8, f16x8>::type;
  using E = typename std::conditional<EL == 0, __bf16, _Float16>::type;
  const unsigned g = blockIdx.x * 512 + threadIdx.x;
  V8 a[4], b[4];
  for (int p = 0; p < 4; ++p)
    for (int i = 0; i < 8; ++i) {
      a[p][i] = (E)hval(g * 64 + p * 8 + i);
      b[p][i] = (E)hval(g * 64 + 32 + p * 8 + i);
    }
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  f32x4 acc[4];
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (EL == 0)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[p], b[(p + j) & 3], acc[j], 0, 0, 0);
        else
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[p], b[(p + j) & 3], acc[j], 0, 0, 0);
      }
  }
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][3];
  if (threadIdx.x == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    stamps[2 * blockIdx.x] = t1 - t0;  // vector stores (thread 0's VGPRs)
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
  out[g] = s;
}

template <int EL>
int run(int iters, int reps, int nblk) {
  float* out;
  unsigned long long* st;
  CHECK(hipMalloc(&out, sizeof(float) * nblk * 512));
  CHECK(hipMalloc(&st, sizeof(unsigned long long) * 2 * nblk));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double fl = 8.0 * nblk * iters * 16 * 16384.0;  // 8 waves x iters x 16 MFMAs of 16 K FLOP
  hipLaunchKernelGGL((mfma_loop<EL>), dim3(nblk), dim3(512), 0, 0, out, st, iters);  // warm-up
  CHECK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((mfma_loop<EL>), dim3(nblk), dim3(512), 0, 0, out, st, iters);
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
    const double ghz = cyc / (real / 100e6) / 1e9;
    printf("{\"dtype\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"frac_2500\": %.4f, \"core_ghz\": %.3f}\n",
           EL ? "fp16" : "bf16", r, ms, fl / ms / 1e9, fl / ms / 1e9 / 2500.0, ghz);
    fflush(stdout);
  }
  CHECK(hipFree(out));
  CHECK(hipFree(st));
  return 0;
}

int main() {
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  for (int pass = 0; pass < 3; ++pass) {  // alternated, so a drifting clock shows in both
    if (run<0>(60000, 2, ncu)) return 1;
    if (run<1>(60000, 2, ncu)) return 1;
  }
  return 0;
}
