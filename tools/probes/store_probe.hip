// Store-bandwidth probe: what a plain 16-B-per-lane store stream reaches on this GPU for the
// env render kernel's sizes (29 MB / 116 MB per launch), back to back, hipEvent timed.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void store_kernel(uint4* p, size_t n16, unsigned v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(v, v, v, v);
}
// per-block contiguous frames: block b writes frames [b*E, (b+1)*E) of HW bytes each
__global__ void frame_kernel(uint8_t* p, int HW, int E, int B, unsigned v) {
  const int chunks = HW / 16;
  for (int e = 0; e < E; ++e) {
    const size_t gb = (size_t)blockIdx.x * E + e;
    if (gb >= (size_t)B) return;
    for (int c = threadIdx.x; c < chunks; c += blockDim.x)
      *reinterpret_cast<uint4*>(p + gb * HW + c * 16) = make_uint4(v, v, v, v);
  }
}

int main() {
  const int B = 4096, HW = 7056;
  for (int mult : {1, 4}) {
    const int b = B * mult;
    size_t bytes = (size_t)b * HW;
    uint8_t* p;
    hipMalloc(&p, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int grid : {1024, 2048, 4096, 8192}) {
      for (int w = 0; w < 5; ++w) store_kernel<<<grid, 256>>>((uint4*)p, bytes / 16, w);
      hipEventRecord(e0);
      for (int w = 0; w < 50; ++w) store_kernel<<<grid, 256>>>((uint4*)p, bytes / 16, w);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      printf("flat  B=%d %6.1f MB grid %d: %.2f us  %.0f GB/s\n", b, bytes / 1e6, grid, ms * 1e3 / 50, bytes / (ms * 1e-3 / 50) / 1e9);
    }
    for (int E : {1, 2, 4}) {
      int grid = (b + E - 1) / E;
      for (int w = 0; w < 5; ++w) frame_kernel<<<grid, 256>>>(p, HW, E, b, w);
      hipEventRecord(e0);
      for (int w = 0; w < 50; ++w) frame_kernel<<<grid, 256>>>(p, HW, E, b, w);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      printf("frame B=%d E=%d: %.2f us  %.0f GB/s\n", b, E, ms * 1e3 / 50, bytes / (ms * 1e-3 / 50) / 1e9);
    }
    hipFree(p);
  }
  return 0;
}
