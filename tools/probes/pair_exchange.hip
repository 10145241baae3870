// Config 2's CU-pair channel split, priced before building it. At 1 024 envs a tower conv is
// bound by each CU streaming the whole 1.18 MB conv pack from L2 (14.8 us per conv). Splitting a quad's
// 256 output channels over two CUs of one XCD halves that stream, but every conv then has to hand each CU's 128-channel
// half of the output (4 envs x 20 px x 128 ch x bf16 = 20 KB) to its partner before the next conv can read all 256
// input channels. This probe runs exactly that per-conv pattern on every CU for one 28-conv tower and times it:
//   stream   each workgroup streams its 0.59 MB half of a conv pack from L2 into registers (8 waves, 16-B loads)
//   exchange each workgroup stores its 20 KB half (16-B sc1 stores), every storing wave waits vmcnt(0), barrier, one
//            lane stores an sc1 flag; the partner polls it (sc1 loads, s_sleep), barrier, then loads the 20 KB (16-B
//            sc1 loads) into LDS — the hand-off of MI355X_MICROARCH.md's 'handoff-flag' / 'handoff-payload' rows,
//            the form whose sc1 loads may replace the acquire
//   both     stream, then exchange (the split conv's critical path if nothing overlaps)
// Workgroups b and b ^ 8 are partners (blocks b and b + 8 share an XCD). The poll gives up after 2^20 tries and
// counts a timeout (so a workgroup that is not resident cannot hang the grid); the launch needs one workgroup per CU.
// Per workgroup, wave 0 stamps s_memtime / s_memrealtime around the 28 convs.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/pair_exchange.hip -o tools/probes/pair_exchange && ./tools/probes/pair_exchange
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
constexpr int NT = 512, CONVS = 28;
constexpr int HALF_PACK = 256 * 9 * 128 * 2;   // 0.59 MB: 128 output channels x 2304 bf16
constexpr int XMAX = 8 * 20 * 128 * 2;         // 40 KB: 8 envs x 20 px x 128 channels bf16 (4 envs: 20 KB)
constexpr int FLAG_STRIDE = 32;                 // ints: one 128-B line per flag

__device__ __forceinline__ void st_sc1(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ u32x4 ld_sc1(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void st_flag(int* p, int v) {
  asm volatile("global_store_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ int ld_flag(const int* p) {
  int v;
  asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// MODE bit 0: stream the half pack, bit 1: exchange XBYTES, bit 2: stream the whole pack (today's per-CU stream)
template <int MODE, int XBYTES>
__global__ __launch_bounds__(NT, 1) void pair_kernel(const u32x4* pack, u32x4* xbuf, int* flags, int epoch,
                                                     unsigned* sink, unsigned long long* stamps, int* timeouts) {
  __shared__ u32x4 stage[XMAX / 16];
  const int b = blockIdx.x, partner = b ^ 8, tid = threadIdx.x;
  unsigned acc = 0;
  unsigned long long t0 = 0, r0 = 0;
  if (tid == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int c = 0; c < CONVS; ++c) {
    if (MODE & 5) {  // this CU's half (or all) of conv c's weight pack (consecutive convs' packs, 33 MB per tower)
      constexpr int NB = (MODE & 4) ? 2 * HALF_PACK : HALF_PACK;
      const u32x4* src = pack + ((size_t)c * 2 * HALF_PACK + ((MODE & 4) ? 0 : (size_t)(b & 1) * HALF_PACK)) / 16;
#pragma unroll 8
      for (int i = tid; i < NB / 16; i += NT) {
        const u32x4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
    if (MODE & 2) {
      u32x4* mine = xbuf + (size_t)b * (XMAX / 16);
      for (int i = tid; i < XBYTES / 16; i += NT) st_sc1(mine + i, u32x4{(unsigned)c, (unsigned)i, (unsigned)b, acc});
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int tag = epoch * 64 + c + 1;
      if (tid == 0) st_flag(flags + b * FLAG_STRIDE, tag);
      if (tid == 0) {
        int n = 0;
        while (ld_flag(flags + partner * FLAG_STRIDE) < tag && ++n < (1 << 20)) __builtin_amdgcn_s_sleep(1);
        if (n >= (1 << 20)) atomicAdd(timeouts, 1);
      }
      __syncthreads();
      const u32x4* theirs = xbuf + (size_t)partner * (XMAX / 16);
      for (int i = tid; i < XBYTES / 16; i += NT) stage[i] = ld_sc1(theirs + i);
      __syncthreads();
      acc ^= stage[(tid * 7 + c) % (XBYTES / 16)].x;
      __syncthreads();  // the partner's next stores overwrite nothing this CU still reads: they go to ITS buffer
    }
  }
  if (tid == 0) {
    stamps[2 * b] = __builtin_amdgcn_s_memtime() - t0;
    stamps[2 * b + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  sink[b * NT + tid] = acc;
}

template <int MODE, int XBYTES>
int run(const char* name, int nblk, const u32x4* pack, u32x4* xbuf, int* flags, unsigned* sink,
        unsigned long long* st, int* to, int& epoch, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < reps; ++r) {
    ++epoch;
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((pair_kernel<MODE, XBYTES>), dim3(nblk), dim3(NT), 0, 0, pack, xbuf, flags, epoch, sink, st, to);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(2 * nblk);
    CHECK(hipMemcpy(h.data(), st, sizeof(unsigned long long) * 2 * nblk, hipMemcpyDeviceToHost));
    int nto = 0;
    CHECK(hipMemcpy(&nto, to, sizeof(int), hipMemcpyDeviceToHost));
    double cyc = 0, real = 0, rmax = 0;
    for (int i = 0; i < nblk; ++i) {
      cyc += h[2 * i];
      real += h[2 * i + 1];
      rmax = h[2 * i + 1] > rmax ? h[2 * i + 1] : rmax;
    }
    const double us_per_conv = (real / nblk) / 100.0 / CONVS;  // s_memrealtime: 100 MHz
    printf("{\"mode\": \"%s\", \"rep\": %d, \"launch_ms\": %.3f, \"us_per_conv_mean_wg\": %.3f, "
           "\"us_per_conv_slowest_wg\": %.3f, \"core_ghz\": %.3f, \"timeouts\": %d}\n",
           name, r, ms, us_per_conv, rmax / 100.0 / CONVS, cyc / (real / 100e6) / 1e9, nto);
    fflush(stdout);
  }
  return 0;
}

int main() {
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int nblk = ncu / 16 * 16;  // whole groups of 16 (pairs b, b ^ 8), one workgroup per CU
  u32x4 *pack, *xbuf;
  int *flags, *to;
  unsigned* sink;
  unsigned long long* st;
  const size_t pack_bytes = (size_t)CONVS * 2 * HALF_PACK;  // 33 MB, the tower's packs
  CHECK(hipMalloc(&pack, pack_bytes));
  CHECK(hipMemset(pack, 1, pack_bytes));
  CHECK(hipMalloc(&xbuf, (size_t)nblk * XMAX));
  CHECK(hipMalloc(&flags, sizeof(int) * nblk * FLAG_STRIDE));
  CHECK(hipMemset(flags, 0, sizeof(int) * nblk * FLAG_STRIDE));
  CHECK(hipMalloc(&to, sizeof(int)));
  CHECK(hipMemset(to, 0, sizeof(int)));
  CHECK(hipMalloc(&sink, sizeof(unsigned) * nblk * NT));
  CHECK(hipMalloc(&st, sizeof(unsigned long long) * 2 * nblk));
  int epoch = 0;
  for (int pass = 0; pass < 2; ++pass) {
    if (run<4, 0>("stream_full_pack", nblk, pack, xbuf, flags, sink, st, to, epoch, 3)) return 1;
    if (run<1, 0>("stream_half_pack", nblk, pack, xbuf, flags, sink, st, to, epoch, 3)) return 1;
    if (run<2, 20480>("exchange_20KB", nblk, pack, xbuf, flags, sink, st, to, epoch, 3)) return 1;
    if (run<2, 40960>("exchange_40KB", nblk, pack, xbuf, flags, sink, st, to, epoch, 3)) return 1;
    if (run<3, 20480>("stream_half+exchange_20KB", nblk, pack, xbuf, flags, sink, st, to, epoch, 3)) return 1;
    if (run<3, 40960>("stream_half+exchange_40KB", nblk, pack, xbuf, flags, sink, st, to, epoch, 3)) return 1;
  }
  return 0;
}
