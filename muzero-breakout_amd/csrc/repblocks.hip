// The representation's residual blocks at 16x20 x 256 channels (networks.py:73-82, ResidualBlock
// :19-35; the trunk's last stage before the first AvgPool2d) in ONE launch, bf16, gfx950 MFMA. The
// stem, the 128-channel blocks and the widening conv before them stay on the band kernels (band.hip), the
// tail (pool, 8x10 blocks, pool, _scale_state) on rep_tail_kernel.
//
// One workgroup (4 waves, one per SIMD) owns ONE env: its 16 x 20 x 256 activation image is 160 KiB,
// the CU's whole LDS, so it stays resident across every conv of the blocks (band_res_kernel re-stages a
// 10-column band with its halo per block and recomputes the halo columns of conv1). A 16-row MFMA tile
// is one image column x (rows = y): a tap (dy, dx) maps tile x onto tile x + dx whole (the 2 tile-taps
// that leave the image are not issued) and shifts rows by dy inside the tile; the one row a shift
// pushes out of the image is zeroed in the B fragment (v_cndmask on the lane that reads it: LDS has no
// room for zero rows). LDS row of (x, y) = 16 x + y (512 B), 16-B chunks XOR-swizzled by y: every B
// fragment read is conflict-free for every shift.
//
// Each conv runs towerp_kernel's structure: the wave's 4 output column tiles in two passes of two (32
// channels x all 20 column tiles = 160 accumulators), the first pass's output held packed in registers,
// weights (the tower packing, agent.pack_tower_conv) through a two-step ring that runs across passes
// and convs, in place (k loops, barrier, write-back, barrier); conv1 lifts the block input at its output
// positions into registers for conv2. Per accumulator the taps are added in the band kernels' order (dy,
// channel step, then dx = 0, -1, +1; their padding taps add exact zeros, skipped or zeroed here); the
// accumulators start at bias (+ residual) as in towerp_kernel, where band_res_kernel adds them after the
// taps (with its epilogue order this kernel equals band_res_kernel bit for bit, but the residual of
// conv2's second pass then stays live through both passes and spills: 8 % slower). Parity: a plain torch
// fp32 evaluation of the bf16-rounded operands, as the band kernels (tests/test_gpu_repblocks.py).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

namespace rf {
constexpr int H = 16, W = 20;          // image rows (a column tile) x columns (tiles)
constexpr int NT = 256;                // 4 waves
constexpr int IMG = 163840;            // 320 rows x 512 B: the CU's LDS
MZ_DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
MZ_DEV float lo(uint32_t u) { return __uint_as_float(u << 16); }
MZ_DEV float hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
MZ_DEV uint32_t relu_pk(uint32_t u) {  // ReLU on two packed bf16 (== the f32 ReLU before rounding)
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(u));
  return r;
}
MZ_DEV uint2 pack(const f32x4& a, bool relu) {
  const uint32_t x = pack_bf16x2(a[0], a[1]), y = pack_bf16x2(a[2], a[3]);
  return relu ? make_uint2(relu_pk(x), relu_pk(y)) : make_uint2(x, y);
}
}  // namespace rf

struct RFArgs {
  const bf16_t* in;  // [B][320][256] NHWC, the blocks' input
  bf16_t* out;       // [B][320][256] NHWC
  const uint4* wf;   // 2 nblocks convs in the tower packing back to back (+ the ring's 8 KB overrun)
  const float* bias; // [2 nblocks][256], BN folded
  int B, nblocks;
};
constexpr int RF_CIN = 256, RF_TNS = 72;                     // every conv 256 -> 256, 3x3
constexpr size_t RF_WCONV = (size_t)16 * RF_TNS * 64;        // uint4 per conv pack

// A wave's view of one pass of a conv: the pack at the pass's first column tile, bytes per column tile,
// channel steps per tap (k step s of the pass, column shift index d = dx + 1: pack step 3 nc d + s)
struct RFW {
  __amdgpu_buffer_rsrc_t rs;
  int ts, nc;
};
MZ_DEV RFW rfw(const uint4* pack, int ct) {
  const uint4* p = pack + (size_t)ct * RF_TNS * 64;
  return RFW{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(p), 0, 0x7fffffff, 0x00020000), RF_TNS * 1024,
             RF_CIN / 32};
}

// B-fragment addressing of lane (q, n) for row shift dy over an image at src with row bytes 1 << rbl:
// byte offset of its row in column 0 (the clamped row for the lane a shift pushes out) and the
// swizzle key; ok = the row is inside the image
MZ_DEV void rf_rows(int src, int rbl, int n, int dy, int& base, int& key, bool& ok) {
  const int yy = n + dy;
  ok = (unsigned)yy < (unsigned)rf::H;
  const int yc = ok ? yy : n;
  base = src + (yc << rbl);
  key = yc;
}

// the 3 nc k steps of one pass with row shift dy = DYI - 1: per (dy, channel step c) the 20 columns in
// 4 groups of 5; a group's 5 B fragments (read during the previous group's first MFMAs) feed dx = 0
// (output x'), dx = -1 (x' + 1) and dx = +1 (x' - 1) of both column tiles. fa holds the first group's
// fragments on entry and the next dy's first on exit.
template <int DYI>
__device__ __forceinline__ void rf_dy(const uint8_t* __restrict__ lds, int src, int rbl, int q, int n, const RFW& cur,
                                      const RFW& nxt, uint4 (&bq)[2][3][2], f32x4 (&acc)[rf::W][2], bf16x8 (&fa)[5],
                                      bf16x8 (&fb)[5], int lane) {
  constexpr int DY = DYI - 1, DYN = DYI == 2 ? -1 : DY + 1;  // the next dy loop's (after dy = +1: the next pass's)
  const int nc = cur.nc, ncp = nc >> 1, cstr = 16 << rbl;
  int base, key, nbase, nkey;
  bool ok, nok;
  rf_rows(src, rbl, n, DY, base, key, ok);
  rf_rows(src, rbl, n, DYN, nbase, nkey, nok);
  (void)nok;
#pragma unroll 1
  for (int cp = 0; cp < ncp; ++cp) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int c = 2 * cp + cc, s = nc * DYI + c;
      const bool wrap = cc == 1 && cp == ncp - 1;  // the next k step opens the next dy loop
      const int xc = base + (((4 * c + q) ^ key) << 4);
      const int xn = wrap ? nbase + ((q ^ nkey) << 4) : base + (((4 * (c + 1) + q) ^ key) << 4);
      // ring slots of this step reload k step s + 2 (past the pass: the next pass's s + 2 - 3 nc)
      int st = s + 2, ts = cur.ts, sn = 3 * nc;
      __amdgpu_buffer_rsrc_t rs = cur.rs;
      if (DYI == 2) {
        const bool past = st >= 3 * nc;
        rs = past ? nxt.rs : cur.rs;
        st = past ? st - 3 * nc : st;
        ts = past ? nxt.ts : cur.ts;
        sn = past ? 3 * nxt.nc : sn;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nb = g < 3 ? xc + 5 * (g + 1) * cstr : xn;
        const bool last = g == 3;
        auto grp = [&](const bf16x8(&f0)[5], bf16x8(&fn)[5]) {
          // every accumulator takes its taps in the band kernels' order dx = 0, -1, +1 within a (dy,
          // channel step): so column 5g's dx = -1 tap (source 5g - 1, the previous group's last
          // fragment, still in fn until this group's read replaces it) comes after its dx = 0 here, and
          // column 5g - 1's dx = +1 tap (source 5g) is issued in this group, after its other two
          bf16x8 f[5], fp;
#pragma unroll
          for (int j = 0; j < 5; ++j) f[j] = (DY == 0 || ok) ? f0[j] : bf16x8{};
          fp = (DY == 0 || ok) ? fn[4] : bf16x8{};
#pragma unroll
          for (int ct = 0; ct < 2; ++ct) {
            const bf16x8 w0 = __builtin_bit_cast(bf16x8, bq[cc][0][ct]);
            const bf16x8 w1 = __builtin_bit_cast(bf16x8, bq[cc][1][ct]);
            const bf16x8 w2 = __builtin_bit_cast(bf16x8, bq[cc][2][ct]);
#pragma unroll
            for (int j = 0; j < 5; ++j) acc[5 * g + j][ct] = rf::mfma(w1, f[j], acc[5 * g + j][ct]);
            if (g > 0) acc[5 * g][ct] = rf::mfma(w0, fp, acc[5 * g][ct]);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[5 * g + j + 1][ct] = rf::mfma(w0, f[j], acc[5 * g + j + 1][ct]);
            if (g > 0) acc[5 * g - 1][ct] = rf::mfma(w2, f[0], acc[5 * g - 1][ct]);
#pragma unroll
            for (int j = 1; j < 5; ++j) acc[5 * g + j - 1][ct] = rf::mfma(w2, f[j], acc[5 * g + j - 1][ct]);
            if (ct == 0) {
#pragma unroll
              for (int j = 0; j < 5; ++j) fn[j] = *reinterpret_cast<const bf16x8*>(lds + nb + j * cstr);
            }
            if (last) {
#pragma unroll
              for (int d = 0; d < 3; ++d)
                bq[cc][d][ct] = __builtin_bit_cast(
                    uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, ct * ts + (sn * d + st) * 1024, 0));
            }
            // the next group's 5 reads ride in column tile 0's MFMA slots 5-9 (fp is a copy of the
            // previous group's last fragment taken before its register is reloaded)
            if (ct == 0) {
              __builtin_amdgcn_sched_group_barrier(0x008, 5, 0);
#pragma unroll
              for (int j = 0; j < 5; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              }
            }
            if (last) __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        };
        if (((cc * 4 + g) & 1) == 0)
          grp(fa, fb);
        else
          grp(fb, fa);
      }
    }
  }
}

MZ_DEV void rf_first_frags(const uint8_t* __restrict__ lds, int src, int rbl, int q, int n, bf16x8 (&fa)[5]) {
  int base, key;
  bool ok;
  rf_rows(src, rbl, n, -1, base, key, ok);
  const int x0 = base + ((q ^ key) << 4), cstr = 16 << rbl;
#pragma unroll
  for (int j = 0; j < 5; ++j) fa[j] = *reinterpret_cast<const bf16x8*>(lds + x0 + j * cstr);
}

// accumulator init of one column of a pass: bias (+ the residual: 4 bf16 channels of the lane's row),
// as towerp_kernel (the band kernels add bias and residual after the taps instead: the sums round
// differently, both within the f32 tolerance of a plain torch evaluation)
MZ_DEV void rf_init1(f32x4 (&acc)[2], const float4 (&b)[2], const uint2 (&res)[2], bool add_res) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    f32x4 v = {b[ct].x, b[ct].y, b[ct].z, b[ct].w};
    if (add_res) {
      const uint2 r = res[ct];
      v[0] += rf::lo(r.x); v[1] += rf::hi(r.x);
      v[2] += rf::lo(r.y); v[3] += rf::hi(r.y);
    }
    acc[ct] = v;
  }
}
MZ_DEV void rf_pin(f32x4 (&acc)[rf::W][2]) {
#pragma unroll
  for (int x = 0; x < rf::W; ++x)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) asm volatile("" : "+a"(acc[x][ct]));
}

// the lane's bias values of pass h of conv k (its column tiles 4 wave + 2h, + 1)
MZ_DEV void rf_bias(float4 (&b)[2], const float* bias, int k, int wave, int h, int q) {
  const int ct0 = 4 * wave + 2 * h;
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) b[ct] = *reinterpret_cast<const float4*>(bias + k * 256 + 16 * (ct0 + ct) + 4 * q);
}

// One pass (h) of conv k: k loops over the pass's two column tiles (acc initialised and pinned by the
// caller), the ring's continuation pointed at the next pass's weights
__device__ __forceinline__ void rf_pass(const RFArgs& a, const uint8_t* __restrict__ lds, int k, int h,
                                        float4 (&bc)[2], uint4 (&bq)[2][3][2], f32x4 (&acc)[rf::W][2],
                                        bf16x8 (&fa)[5], bf16x8 (&fb)[5], int lane, int wave) {
  const int q = lane >> 4, n = lane & 15;
  // the next pass: this conv's second, the next conv's first, or (after the last) this one again
  // (loads in range, never used); its bias now, its weights by the ring
  const int nconv = 2 * a.nblocks;
  const bool more = h == 0, nextk = !more && k + 1 < nconv;
  const int nk = more ? k : (nextk ? k + 1 : k), nh = more ? 1 : 0;
  (void)bc;
  const RFW cur = rfw(a.wf + k * RF_WCONV, 4 * wave + 2 * h);
  const RFW nxt = (more || nextk) ? rfw(a.wf + nk * RF_WCONV, 4 * wave + 2 * nh) : cur;
  rf_dy<0>(lds, 0, 9, q, n, cur, nxt, bq, acc, fa, fb, lane);
  rf_dy<1>(lds, 0, 9, q, n, cur, nxt, bq, acc, fa, fb, lane);
  rf_dy<2>(lds, 0, 9, q, n, cur, nxt, bq, acc, fa, fb, lane);
}

// One conv of a block, k loops then an in-place write-back. RES false: conv1 (the write-back first
// lifts the block input at the wave's output positions into res); true: conv2 (acc starts at bias +
// res). ReLU on both. bc: this conv's pass-0 bias on entry, the next conv's on exit (every bias loaded
// a pass ahead of its use).
template <bool RES>
__device__ __forceinline__ void rf_conv(const RFArgs& a, uint8_t* __restrict__ lds, int k, float4 (&bc)[2],
                                        uint2 (&res)[2][rf::W][2], uint4 (&bq)[2][3][2], int lane, int wave) {
  const int q = lane >> 4, n = lane & 15;
  bf16x8 fa[5], fb[5];
  rf_first_frags(lds, 0, 9, q, n, fa);
  uint2 out0[rf::W][2];
  f32x4 acc[rf::W][2];
#pragma unroll
  for (int x = 0; x < rf::W; ++x) rf_init1(acc[x], bc, res[0][x], RES);
  rf_pin(acc);
  rf_bias(bc, a.bias, k, wave, 1, q);  // pass 1's bias, ahead of pass 0's k loop
  rf_pass(a, lds, k, 0, bc, bq, acc, fa, fb, lane, wave);
#pragma unroll
  for (int x = 0; x < rf::W; ++x) {  // pass 0 out (ReLU, bf16, held), pass 1 in, column by column
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) out0[x][ct] = rf::pack(acc[x][ct], true);
    rf_init1(acc[x], bc, res[1][x], RES);
    __builtin_amdgcn_sched_barrier(0);
  }
  rf_pin(acc);
  rf_bias(bc, a.bias, k + 1 < 2 * a.nblocks ? k + 1 : k, wave, 0, q);  // the next conv's pass-0 bias
  rf_pass(a, lds, k, 1, bc, bq, acc, fa, fb, lane, wave);
  __syncthreads();  // every wave has read the whole image
  // write-back column by column: row 16 x + n (swizzle key n), the wave's 64 channels. The lane's
  // offsets are recomputed per conv from an opaque copy of n: left CSE'd across the block's convs, the
  // 80 addresses stayed live through conv2 and were spilled, each reload waiting on the weight ring
  int no = n;
  asm volatile("" : "+v"(no));
  int cofs[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int ch = 16 * (4 * wave + ct) + 4 * q;
    cofs[ct] = (no << 9) + (((ch >> 3) ^ no) << 4) + ((ch & 7) << 1);
  }
#pragma unroll
  for (int x = 0; x < rf::W; ++x) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      uint2* p = reinterpret_cast<uint2*>(lds + (x << 13) + cofs[ct]);
      if (!RES) res[ct >> 1][x][ct & 1] = *p;
      *p = ct < 2 ? out0[x][ct] : rf::pack(acc[x][ct - 2], true);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
}

__global__ __launch_bounds__(rf::NT, 1) void rep_blocks_kernel(RFArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[rf::IMG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4;
  const int b = blockIdx.x;
  uint4 bq[2][3][2];
  {  // the ring's first two k steps (conv 0, pass 0)
    const RFW w0 = rfw(a.wf, 4 * wave);
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
          bq[cc][d][ct] = __builtin_bit_cast(
              uint4, __builtin_amdgcn_raw_buffer_load_b128(w0.rs, lane * 16, ct * w0.ts + (3 * w0.nc * d + cc) * 1024, 0));
  }
  float4 bc[2];
  rf_bias(bc, a.bias, 0, wave, 0, q);
  {  // stage: pixel p = 20 y + x -> LDS row 16 x + y, two batches of 20 chunks per thread
    const bf16_t* src = a.in + (size_t)b * rf::H * rf::W * 256;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      uint4 v[20];
#pragma unroll
      for (int u = 0; u < 20; ++u) v[u] = *reinterpret_cast<const uint4*>(src + (size_t)((hb * 20 + u) * rf::NT + tid) * 8);
#pragma unroll
      for (int u = 0; u < 20; ++u) {
        const int i = (hb * 20 + u) * rf::NT + tid, p = i >> 5, c = i & 31, y = p / rf::W, x = p % rf::W;
        *reinterpret_cast<uint4*>(lds + ((x * 16 + y) << 9) + ((c ^ y) << 4)) = v[u];
      }
    }
  }
  __syncthreads();
  for (int blk = 0; blk < a.nblocks; ++blk) {
    uint2 res[2][rf::W][2];  // lives from conv1's write-back to conv2's inits
    rf_conv<false>(a, lds, 2 * blk, bc, res, bq, lane, wave);
    rf_conv<true>(a, lds, 2 * blk + 1, bc, res, bq, lane, wave);
  }
  // the output, NHWC: pixel p = 20 y + x from LDS row 16 x + y
  bf16_t* dst = a.out + (size_t)b * rf::H * rf::W * 256;
#pragma unroll 4
  for (int u = 0; u < 40; ++u) {
    const int i = u * rf::NT + tid, p = i >> 5, c = i & 31, y = p / rf::W, x = p % rf::W;
    *reinterpret_cast<uint4*>(dst + (size_t)i * 8) =
        *reinterpret_cast<const uint4*>(lds + ((x * 16 + y) << 9) + ((c ^ y) << 4));
  }
}

}  // namespace

extern "C" {

// nblocks ResidualBlock(256) at 16x20 in one launch (see above): in / out [B][320][256] bf16 NHWC
// (distinct buffers), wf16: the 2 nblocks convs in the tower packing back to back + 8 KB, bias
// [2 nblocks][256] f32 (BN folded)
int mzba_rep_blocks(const void* in, void* out, const void* wf16, const float* bias, int nblocks, int B,
                    hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nblocks >= 1 && nblocks <= 24 && in && out && wf16 && bias && in != out, -1);
  RFArgs a{(const bf16_t*)in, (bf16_t*)out, (const uint4*)wf16, bias, B, nblocks};
  hipLaunchKernelGGL(rep_blocks_kernel, dim3(B), dim3(rf::NT), 0, stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
