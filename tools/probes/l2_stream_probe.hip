// Per-CU weight-stream probe for config 2's bound: every workgroup (one per CU, 4 waves) streams
// the whole 14-block tower pack (28 convs x 16 column tiles x 72 k steps x 1 KB = 33 MB) in the tower kernels'
// order and access form — buffer_load_dwordx4 off a wave-uniform resource, each wave its 4 column tiles, D loads
// in flight per wave — and does nothing else with it (an XOR keeps the data live). 256 workgroups = all CUs, as
// tower8_kernel<0, 1> runs config 2's 1 024 envs. Reports the per-CU rate (the whole pack per CU / launch time)
// for ring depths D, which bounds a conv at: 1.18 MB of weights per CU per conv / that rate.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/probes/l2_stream_probe tools/probes/l2_stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NCONV = 28, NCT = 16, NS = 72, FRAG = 1024;

template <int D>
__global__ __launch_bounds__(256, 1) void wstream(const uint4* pack, unsigned* sink, int nconv) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(pack), 0, 0x7fffffff, 0x00020000);
  // fragment f of the wave's stream: conv f / (4 NS), column tile 4 wave + f % 4, k step (f / 4) % NS
  auto off = [&](int f) {
    const int conv = f / (4 * NS), r = f % (4 * NS), s = r / 4, ct = 4 * wave + (r & 3);
    return (conv * NCT * NS + ct * NS + s) * FRAG;
  };
  const int nf = nconv * 4 * NS;
  uint4 ring[D];
  uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < D; ++i)
    ring[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, off(i), 0));
  for (int f0 = 0; f0 < nf; f0 += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      acc.x ^= ring[i].x; acc.y ^= ring[i].y; acc.z ^= ring[i].z; acc.w ^= ring[i].w;
      const int f = f0 + D + i;
      ring[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, off(f < nf ? f : 0), 0));
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc.x;  // never true in practice
}

template <int D>
void run(const uint4* pack, unsigned* sink, int grid, const char* tag) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 5; ++w) wstream<D><<<grid, 256>>>(pack, sink, NCONV);
  const int it = 20;
  hipEventRecord(e0);
  for (int w = 0; w < it; ++w) wstream<D><<<grid, 256>>>(pack, sink, NCONV);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / it, per_cu = (double)NCONV * NCT * NS * FRAG;
  printf("{\"probe\": \"l2_weight_stream\", \"ring_depth_per_wave\": %d, \"grid\": %d, \"launch_us\": %.2f, "
         "\"bytes_per_cu\": %.0f, \"per_cu_GBps\": %.1f, \"chip_GBps\": %.0f, \"conv_floor_us\": %.3f, \"tag\": \"%s\"}\n",
         D, grid, us, per_cu, per_cu / (us * 1e-6) / 1e9, per_cu * grid / (us * 1e-6) / 1e9, us / NCONV, tag);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  const size_t bytes = (size_t)NCONV * NCT * NS * FRAG + 8 * 64 * 16;
  uint4* pack;
  unsigned* sink;
  hipMalloc(&pack, bytes);
  hipMalloc(&sink, 4096);
  hipMemset(pack, 0x3c, bytes);
  for (int grid : {256, 128, 64}) {
    run<6>(pack, sink, grid, "tower8 ring (6 per wave)");
    run<12>(pack, sink, grid, "12 per wave");
    run<24>(pack, sink, grid, "24 per wave");
  }
  hipFree(pack);
  hipFree(sink);
  return 0;
}
