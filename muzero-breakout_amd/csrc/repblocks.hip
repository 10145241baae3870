// The representation's trunk at 16x20 (networks.py:46-82: the stem Conv2d(2L -> c0), the c0-channel
// ResidualBlocks, the widening Conv2d(c0 -> c1), the c1-channel ResidualBlocks; ResidualBlock :19-35)
// in ONE launch, bf16, gfx950 MFMA — everything before the first AvgPool2d. The tail (pool, 8x10 blocks,
// pool, _scale_state) runs on rep_tail_kernel. The same kernel without its stem stage is
// mzba_rep_blocks (the c1 = 256-channel blocks alone).
//
// One workgroup (4 waves, one per SIMD) owns ONE env: its 16 x 20 activation image (64, 128 or 256
// channels: 40 / 80 / 160 KiB, the last the CU's whole LDS) stays resident from the staged input to the
// last block (the band kernels re-stage a 10-column band with its halo per conv or block and recompute the
// halo columns). A 16-row MFMA tile is one image column x (rows = y): a tap (dy, dx) maps tile x onto tile
// x + dx whole (the 2 tile-taps that leave the image are not issued) and shifts rows by dy inside the tile;
// the one row a shift pushes out of the image is zeroed in the B fragment (v_cndmask on the lane that
// reads it: LDS has no room for zero rows; that lane reads row (y + dy) & 15 of the column, whose key
// completes its bank group). LDS row of (x, y) = 16 x + y (2C bytes), 16-B chunks XOR-swizzled by a key
// of y (rf::key below): every B fragment read is conflict-free for every shift.
//
// Each conv runs towerp_kernel's structure: a wave owns a quarter of the output channels (32 at Cout 128:
// one pass of two column tiles; 64 at Cout 256: two passes, the first pass's output held packed in
// registers), all 20 column tiles (40 accumulators a pass); weights (the tower packing,
// agent.pack_tower_conv) through a two-step ring that runs across passes and convs, whatever their
// widths; in place (k loops, barrier, write-back in the output's row width, barrier — every input read
// precedes every output write, so a conv may widen the image); conv1 of a block lifts the block input
// at its output positions into registers for conv2. Per accumulator the taps are added in the band
// kernels' order (dy, channel step, then dx = 0, -1, +1; their padding taps add exact zeros, skipped or
// zeroed here); the accumulators start at bias (+ residual) as in towerp_kernel, where band_res_kernel
// adds them after the taps (with its epilogue order this kernel equals band_res_kernel bit for bit, but
// the residual of conv2's second pass then stays live through both passes and spills: 8 % slower).
// Parity: a plain torch fp32 evaluation of the bf16-rounded operands, as the band kernels
// (tests/test_gpu_repblocks.py).
#include "common.h"


namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

namespace rf {
constexpr int H = 16, W = 20;          // image rows (a column tile) x columns (tiles)
constexpr int NT = 256;                // 4 waves
constexpr int IMG = 163840;            // 320 rows x 512 B: the CU's LDS
constexpr int MAXC = 56;               // convs per launch (kernel-argument pointer tables)
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
// swizzle key of image row y for rows of 1 << RBL bytes. ds_read_b128 serves a wave in four lane groups
// of 16 (MI355X_MICROARCH.md, LDS table), {0-3, 12-15, 20-27} etc.: a group holds rows n = 0-3, 12-15 of
// one k quarter q and rows 4-11 of quarter q ^ 1, so it is conflict-free when the 16 (bank set of the row
// start + (4c + q) ^ key) values differ for every row shift dy. key = y (round 3) met that at dy = 0 only:
// the two shifted thirds of the reads were 2-way conflicted (SQ_LDS_BANK_CONFLICT 0.41 of LDS-active
// cycles, profiles/r04/r4d). 256- and 512-B rows (every row starts in bank set 0): key = 2 (y & 3) | 9 (y
// bit 2), which keeps any 16 consecutive rows apart (rows y, y + 8 share a key; the wrapped row of an
// out-of-image lane fills its group) and spreads a 16-row ds_write_b64 over all 8 slots of its 128-B
// window (2-way, its minimum); 128-B rows (the stem input, bank set 8 (y & 1) + chunk, 8 chunks): a
// searched table (tools/swizzle_search.py)
template <int RBL> MZ_DEV int key(int y) {
  if (RBL == 7) return (int)((0x7662265544022100ull >> (4 * y)) & 7u);
  return ((y << 1) & 6) | (((y >> 2) & 1) * 9);
}
template <int C> constexpr int rbl() { return C == 64 ? 7 : (C == 128 ? 8 : 9); }
}  // namespace rf

struct RFArgs {
  const bf16_t* in;               // [B][320][Cin] NHWC: 2L = 64 channels with the stem, else 256
  bf16_t* out;                    // [B][320][256] NHWC
  const uint4* w[rf::MAXC];       // per conv: its tower packing (+ the ring's 8 KB overrun after the last)
  const float* b[rf::MAXC];       // per conv: [Cout] f32, BN folded
  int n0, n1, B;                  // c0- / c1-channel blocks; n0 < 0: no stem stage (mzba_rep_blocks)
};
// conv k's widths: with the stem, k = 0 stem (64 -> 128), 1 .. 2 n0 the 128-channel blocks, 2 n0 + 1 the
// widening conv (128 -> 256), then the 256-channel blocks; without it, every conv 256 -> 256
MZ_DEV int rf_cin(const RFArgs& a, int k) { return a.n0 < 0 ? 256 : (k == 0 ? 64 : (k <= 2 * a.n0 + 1 ? 128 : 256)); }
MZ_DEV int rf_cout(const RFArgs& a, int k) { return a.n0 < 0 ? 256 : (k <= 2 * a.n0 ? 128 : 256); }
MZ_DEV int rf_nconv(const RFArgs& a) { return a.n0 < 0 ? 2 * a.n1 : 2 * a.n0 + 2 + 2 * a.n1; }

// A wave's view of one pass of a conv: the pack at the pass's first column tile, bytes per column tile,
// channel steps per tap (k step s of the pass, column shift index d = dx + 1: pack step 3 nc d + s)
struct RFW {
  __amdgpu_buffer_rsrc_t rs;
  int ts, nc;
};
// pass h of conv k for wave `wave`: its column tiles (Cout / 64) wave + 2 h, + 1
MZ_DEV RFW rfw(const RFArgs& a, int k, int wave, int h) {
  const int nc = rf_cin(a, k) / 32, ct = (rf_cout(a, k) / 64) * wave + 2 * h;
  const uint4* p = a.w[k] + (size_t)ct * 9 * nc * 64;
  return RFW{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(p), 0, 0x7fffffff, 0x00020000), 9 * nc * 1024, nc};
}

// B-fragment addressing of lane (q, n) for row shift dy over an image at src with rows of 1 << RBL bytes:
// byte offset of its row in column 0 (the wrapped row for the lane a shift pushes out) and the swizzle
// key; ok = the row is inside the image
template <int RBL>
MZ_DEV void rf_rows(int src, int n, int dy, int& base, int& key, bool& ok) {
  const int yy = n + dy;
  ok = (unsigned)yy < (unsigned)rf::H;
  const int yc = yy & (rf::H - 1);  // out of the image: the wrapped row (read, then zeroed)
  base = src + (yc << RBL);
  key = rf::key<RBL>(yc);
}

// the 3 NC k steps of one pass with row shift dy = DYI - 1: per (dy, channel step c) the 20 columns in
// 4 groups of 5; a group's 5 B fragments (read during the previous group's first MFMAs) feed dx = 0
// (output x'), dx = -1 (x' + 1) and dx = +1 (x' - 1) of both column tiles. fa holds the first group's
// fragments on entry and the next dy's first on exit.
template <int DYI, int RBL, int NC>
__device__ __forceinline__ void rf_dy(const uint8_t* __restrict__ lds, int src, int q, int n, const RFW& cur,
                                      const RFW& nxt, uint4 (&bq)[2][3][2], f32x4 (&acc)[rf::W][2], bf16x8 (&fa)[5],
                                      bf16x8 (&fb)[5], int lane) {
  constexpr int DY = DYI - 1, DYN = DYI == 2 ? -1 : DY + 1;  // the next dy loop's (after dy = +1: the next pass's)
  constexpr int ncp = NC >> 1, cstr = 16 << RBL;
  int base, key, nbase, nkey;
  bool ok, nok;
  rf_rows<RBL>(src, n, DY, base, key, ok);
  rf_rows<RBL>(src, n, DYN, nbase, nkey, nok);
  (void)nok;
#pragma unroll 1
  for (int cp = 0; cp < ncp; ++cp) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int c = 2 * cp + cc, s = NC * DYI + c;
      const bool wrap = cc == 1 && cp == ncp - 1;  // the next k step opens the next dy loop
      const int xc = base + (((4 * c + q) ^ key) << 4);
      const int xn = wrap ? nbase + ((q ^ nkey) << 4) : base + (((4 * (c + 1) + q) ^ key) << 4);
      // ring slots of this step reload k step s + 2 (past the pass: the next pass's s + 2 - 3 NC)
      int st = s + 2, ts = cur.ts, sn = 3 * NC;
      __amdgpu_buffer_rsrc_t rs = cur.rs;
      if (DYI == 2) {
        const bool past = st >= 3 * NC;
        rs = past ? nxt.rs : cur.rs;
        st = past ? st - 3 * NC : st;
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

template <int RBL>
MZ_DEV void rf_first_frags(const uint8_t* __restrict__ lds, int src, int q, int n, bf16x8 (&fa)[5]) {
  int base, key;
  bool ok;
  rf_rows<RBL>(src, n, -1, base, key, ok);
  const int x0 = base + ((q ^ key) << 4), cstr = 16 << RBL;
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

// the lane's bias values of pass h of conv k (its column tiles (Cout / 64) wave + 2h, + 1)
MZ_DEV void rf_bias(float4 (&b)[2], const RFArgs& a, int k, int wave, int h, int q) {
  const int ct0 = (rf_cout(a, k) / 64) * wave + 2 * h;
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) b[ct] = *reinterpret_cast<const float4*>(a.b[k] + 16 * (ct0 + ct) + 4 * q);
}

// One pass (h) of conv k: k loops over the pass's two column tiles (acc initialised and pinned by the
// caller), the ring's continuation pointed at the next pass's weights: this conv's second, the next
// conv's first, or (after the last) this one again (loads in range, never used)
template <int RBL, int NC, int NP>
__device__ __forceinline__ void rf_pass(const RFArgs& a, const uint8_t* __restrict__ lds, int k, int h,
                                        uint4 (&bq)[2][3][2], f32x4 (&acc)[rf::W][2], bf16x8 (&fa)[5],
                                        bf16x8 (&fb)[5], int lane, int wave) {
  const int q = lane >> 4, n = lane & 15;
  const bool more = h + 1 < NP, nextk = !more && k + 1 < rf_nconv(a);
  const RFW cur = rfw(a, k, wave, h);
  const RFW nxt = more ? rfw(a, k, wave, h + 1) : (nextk ? rfw(a, k + 1, wave, 0) : cur);
  rf_dy<0, RBL, NC>(lds, 0, q, n, cur, nxt, bq, acc, fa, fb, lane);
  rf_dy<1, RBL, NC>(lds, 0, q, n, cur, nxt, bq, acc, fa, fb, lane);
  rf_dy<2, RBL, NC>(lds, 0, q, n, cur, nxt, bq, acc, fa, fb, lane);
}

// One conv (Cin -> Cout, 3x3), k loops then an in-place write-back. RES 0: plain (the stem and the
// widening conv: no activation, networks.py:47-55, 64-72); 1: conv1 of a block (ReLU; the write-back
// first lifts the block input at the wave's output positions into res); 2: conv2 (acc starts at bias +
// res, ReLU after the sum). bc: this conv's pass-0 bias on entry, the next conv's on exit (every bias
// loaded a pass ahead of its use).
template <int CIN, int COUT, int RES>
__device__ __forceinline__ void rf_conv(const RFArgs& a, uint8_t* __restrict__ lds, int k, float4 (&bc)[2],
                                        uint2 (&res)[COUT / 128][rf::W][2], uint4 (&bq)[2][3][2], int lane,
                                        int wave) {
  constexpr int RBI = rf::rbl<CIN>(), RBO = rf::rbl<COUT>(), NC = CIN / 32, NP = COUT / 128, CTW = COUT / 64;
  constexpr bool RELU = RES != 0;
  static_assert(RES == 0 || CIN == COUT, "residual blocks keep their width");
  const int q = lane >> 4, n = lane & 15;
  const int kn = k + 1 < rf_nconv(a) ? k + 1 : k;
  bf16x8 fa[5], fb[5];
  rf_first_frags<RBI>(lds, 0, q, n, fa);
  uint2 out0[rf::W][2];  // pass 0's output (two passes only)
  f32x4 acc[rf::W][2];
#pragma unroll
  for (int x = 0; x < rf::W; ++x) rf_init1(acc[x], bc, res[0][x], RES == 2);
  rf_pin(acc);
  if (NP > 1)
    rf_bias(bc, a, k, wave, 1, q);  // pass 1's bias, ahead of pass 0's k loop
  else
    rf_bias(bc, a, kn, wave, 0, q);  // the next conv's pass-0 bias
  rf_pass<RBI, NC, NP>(a, lds, k, 0, bq, acc, fa, fb, lane, wave);
  if constexpr (NP > 1) {
#pragma unroll
    for (int x = 0; x < rf::W; ++x) {  // pass 0 out (bf16, held), pass 1 in, column by column
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) out0[x][ct] = rf::pack(acc[x][ct], RELU);
      rf_init1(acc[x], bc, res[NP - 1][x], RES == 2);
      __builtin_amdgcn_sched_barrier(0);
    }
    rf_pin(acc);
    rf_bias(bc, a, kn, wave, 0, q);  // the next conv's pass-0 bias
    rf_pass<RBI, NC, NP>(a, lds, k, 1, bq, acc, fa, fb, lane, wave);
  }
  __syncthreads();  // every wave has read the whole image
  // write-back column by column: row 16 x + n (swizzle key of n), the wave's Cout / 4 channels. The
  // lane's offsets are recomputed per conv from an opaque copy of n: left CSE'd across the block's convs,
  // the 80 addresses stayed live through conv2 and were spilled, each reload waiting on the weight ring
  int no = n;
  asm volatile("" : "+v"(no));
  int cofs[CTW];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) {
    const int ch = 16 * (CTW * wave + ct) + 4 * q;
    cofs[ct] = (no << RBO) + (((ch >> 3) ^ rf::key<RBO>(no)) << 4) + ((ch & 7) << 1);
  }
#pragma unroll
  for (int x = 0; x < rf::W; ++x) {
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) {
      uint2* p = reinterpret_cast<uint2*>(lds + (x << (RBO + 4)) + cofs[ct]);
      if (RES == 1) res[ct >> 1][x][ct & 1] = *p;
      *p = (NP > 1 && ct < 2) ? out0[x][ct] : rf::pack(acc[x][ct - (NP > 1 ? 2 : 0)], RELU);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
}

// STEM: the input is the 64-channel representation input and the launch runs the whole trunk; else the
// input is the 256-channel image and the launch runs the n1 blocks alone (mzba_rep_blocks)
template <bool STEM>
__global__ __launch_bounds__(rf::NT, 1) void rep_trunk_kernel(RFArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[rf::IMG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4;
  const int b = blockIdx.x;
  uint4 bq[2][3][2];
  {  // the ring's first two k steps (conv 0, pass 0)
    const RFW w0 = rfw(a, 0, wave, 0);
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
  rf_bias(bc, a, 0, wave, 0, q);
  if constexpr (STEM) {  // stage: pixel p = 20 y + x -> LDS row 16 x + y (128 B, key<7>), 10 chunks per thread
    const bf16_t* src = a.in + (size_t)b * rf::H * rf::W * 64;
    uint4 v[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) v[u] = *reinterpret_cast<const uint4*>(src + (size_t)(u * rf::NT + tid) * 8);
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int i = u * rf::NT + tid, p = i >> 3, c = i & 7, y = p / rf::W, x = p % rf::W;
      *reinterpret_cast<uint4*>(lds + ((x * 16 + y) << 7) + ((c ^ rf::key<7>(y)) << 4)) = v[u];
    }
  } else {  // stage: pixel p = 20 y + x -> LDS row 16 x + y, two batches of 20 chunks per thread
    const bf16_t* src = a.in + (size_t)b * rf::H * rf::W * 256;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      uint4 v[20];
#pragma unroll
      for (int u = 0; u < 20; ++u) v[u] = *reinterpret_cast<const uint4*>(src + (size_t)((hb * 20 + u) * rf::NT + tid) * 8);
#pragma unroll
      for (int u = 0; u < 20; ++u) {
        const int i = (hb * 20 + u) * rf::NT + tid, p = i >> 5, c = i & 31, y = p / rf::W, x = p % rf::W;
        *reinterpret_cast<uint4*>(lds + ((x * 16 + y) << 9) + ((c ^ rf::key<9>(y)) << 4)) = v[u];
      }
    }
  }
  __syncthreads();
  int k = 0;
  if constexpr (STEM) {
    {
      uint2 none[1][rf::W][2];
      rf_conv<64, 128, 0>(a, lds, k++, bc, none, bq, lane, wave);
    }
    for (int blk = 0; blk < a.n0; ++blk) {
      uint2 res[1][rf::W][2];  // lives from conv1's write-back to conv2's inits
      rf_conv<128, 128, 1>(a, lds, k++, bc, res, bq, lane, wave);
      rf_conv<128, 128, 2>(a, lds, k++, bc, res, bq, lane, wave);
    }
    {
      uint2 none[2][rf::W][2];
      rf_conv<128, 256, 0>(a, lds, k++, bc, none, bq, lane, wave);
    }
  }
  for (int blk = 0; blk < a.n1; ++blk) {
    uint2 res[2][rf::W][2];  // lives from conv1's write-back to conv2's inits
    rf_conv<256, 256, 1>(a, lds, k++, bc, res, bq, lane, wave);
    rf_conv<256, 256, 2>(a, lds, k++, bc, res, bq, lane, wave);
  }
  // the output, NHWC: pixel p = 20 y + x from LDS row 16 x + y
  bf16_t* dst = a.out + (size_t)b * rf::H * rf::W * 256;
#pragma unroll 4
  for (int u = 0; u < 40; ++u) {
    const int i = u * rf::NT + tid, p = i >> 5, c = i & 31, y = p / rf::W, x = p % rf::W;
    *reinterpret_cast<uint4*>(dst + (size_t)i * 8) =
        *reinterpret_cast<const uint4*>(lds + ((x * 16 + y) << 9) + ((c ^ rf::key<9>(y)) << 4));
  }
}

constexpr size_t RF_WCONV = (size_t)16 * 72 * 64;  // uint4 per 256 -> 256 conv pack

}  // namespace

extern "C" {

// nblocks ResidualBlock(256) at 16x20 in one launch (the trunk kernel without its stem stage): in / out
// [B][320][256] bf16 NHWC (distinct buffers), wf16: the 2 nblocks convs in the tower packing back to
// back + 8 KB, bias [2 nblocks][256] f32 (BN folded)
int mzba_rep_blocks(const void* in, void* out, const void* wf16, const float* bias, int nblocks, int B,
                    hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nblocks >= 1 && nblocks <= 24 && in && out && wf16 && bias && in != out, -1);
  RFArgs a{};
  a.in = (const bf16_t*)in, a.out = (bf16_t*)out, a.n0 = -1, a.n1 = nblocks, a.B = B;
  for (int k = 0; k < 2 * nblocks; ++k) {
    a.w[k] = (const uint4*)wf16 + k * RF_WCONV;
    a.b[k] = bias + k * 256;
  }
  hipLaunchKernelGGL(rep_trunk_kernel<false>, dim3(B), dim3(rf::NT), 0, stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

// the representation trunk at 16x20 in one launch (see above): in [B][320][64] bf16 NHWC (the
// representation input, 2L = 64 channels), out [B][320][256] bf16 NHWC (distinct); w / b: host arrays of
// the 2 n0 + 2 + 2 n1 convs' device pointers in network order (stem 64 -> 128, the n0 blocks' conv1 /
// conv2 at 128, the widening conv 128 -> 256, the n1 blocks' at 256): each weight in the tower packing,
// the last followed by the ring's 8 KB overrun; each bias [Cout] f32 (BN folded into the block convs)
int mzba_rep_trunk(const void* in, void* out, const void* const* w, const float* const* b, int n0, int n1, int B,
                   hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && n0 >= 0 && n1 >= 0 && 2 * n0 + 2 + 2 * n1 <= rf::MAXC && in && out && w && b && in != out, -1);
  RFArgs a{};
  a.in = (const bf16_t*)in, a.out = (bf16_t*)out, a.n0 = n0, a.n1 = n1, a.B = B;
  for (int k = 0; k < 2 * n0 + 2 + 2 * n1; ++k) {
    MZ_CHECK_ARG(w[k] && b[k], -1);
    a.w[k] = (const uint4*)w[k];
    a.b[k] = b[k];
  }
  hipLaunchKernelGGL(rep_trunk_kernel<true>, dim3(B), dim3(rf::NT), 0, stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
