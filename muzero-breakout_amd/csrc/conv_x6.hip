// f32-faithful 3x3 convolution on bf16 MFMAs ("x6": split-bf16 products), for the f32 parity path's
// latent towers (networks.py:19-35, 103-241): the parity path runs the reference's f32 arithmetic, whose
// ceiling on the f32-input MFMA (v_mfma_f32_16x16x4_f32, 157 TF) is 1/16 of the bf16 one.
//
// Every f32 operand is split exactly-rounded into three bf16 parts, x = xh + xm + xl (xh = bf16(x),
// xm = bf16(x - xh), xl = bf16(x - xh - xm); |xm| <= 2^-9 |x|, |xl| <= 2^-18 |x|), and a product is taken
// as the six terms down to the 2^-18 order, xh wh + xh wm + xm wh + xh wl + xm wm + xl wh, each a bf16 x bf16
// MFMA accumulating in f32: the dropped terms (xm wl, xl wm, xl wl) are below 2^-26 of the product and the
// parts' own rounding below 2^-26, so a conv is as close to the exact result as an f32 one (a 14-block tower
// simulated on the CPU: 2.5e-7 of the magnitude from f64, the f32 chain 4.1e-7). Six bf16 MFMAs cost 6/16 of
// one f32 MFMA's issue.
//
// Structure: conv_halo_kernel's (csrc/conv_halo.hip) — a workgroup stages TM consecutive output pixels plus
// W + 1 halo rows on each side once (here the f32 activations: Cin x 4 B per row, 16-B chunks XOR-swizzled
// by row), runs all 9 taps from LDS (taps leaving the image read a 16-row zero block), 8 waves = 2 pixel halves x 4
// output-channel quarters; weights = MFMA A operand, their three bf16 parts pre-split on the host
// (agent.py "wx": three pack_lat16 packs back to back) through a two-k-step register ring; activations = B
// operand, read as f32 from LDS and split in registers per fragment (each split feeds 4 column tiles x 6
// MFMAs). Epilogue in f32: + bias (+ residual), ReLU.
#include "common.h"
#include "elt.h"
#include <type_traits>
#include <utility>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

namespace x6 {
constexpr int TN = 256;            // output channels per workgroup
constexpr int NT = 512;            // 8 waves, two per SIMD
constexpr int LDS_MAX = 160 * 1024;
}  // namespace x6

struct X6Args {
  const float* in;     // [M][Cin] f32
  const bf16_t* wx;    // [3 parts][Cout / 16][9 Cin / 32][64][8] (x3: [2 fp16 parts]...)
  const float* bias;   // [Cout]
  const float* res;    // optional [M][Cout] f32
  float* out;          // [M][Cout] f32
  int M, H, W, Cin, Cout, relu;
  int HALO, NI, ZOFF;  // halo rows each side, LDS-DMA 1-KiB blocks of the staging, byte offset of the zero block
  long long part;      // elements per weight part
  const float* wscale = nullptr;  // x3 (conv_x6p_kernel NP = 2): per output channel 2^-k of the weights' scaling
};

// bf16 split of 8 f32 (two 16-B halves): hi, mid, lo with x == hi + mid + lo up to the lo part's rounding
MZ_DEV void split8(const uint4& u0, const uint4& u1, bf16x8& h, bf16x8& m, bf16x8& l) {
  const float x[8] = {__uint_as_float(u0.x), __uint_as_float(u0.y), __uint_as_float(u0.z), __uint_as_float(u0.w),
                      __uint_as_float(u1.x), __uint_as_float(u1.y), __uint_as_float(u1.z), __uint_as_float(u1.w)};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const __bf16 hb = (__bf16)x[i];
    const float r = x[i] - (float)hb;
    const __bf16 mb = (__bf16)r;
    const float r2 = r - (float)mb;
    h[i] = hb;
    m[i] = mb;
    l[i] = (__bf16)r2;
  }
}

// fp16 split of 8 f32 for the x3 form: hi = fp16(x), lo = fp16(x - hi) (x - hi is exact in f32; |lo| <= 2^-11 |x|,
// lo's own rounding <= 2^-22 |x| while lo is normal, i.e. |x| >= 2^-3; below, absolute 2^-25). |x| < 65520 or
// hi = inf and the output turns non-finite (loud, never silently wrong)
MZ_DEV void split8h(const uint4& u0, const uint4& u1, f16x8& h, f16x8& l) {
  const float x[8] = {__uint_as_float(u0.x), __uint_as_float(u0.y), __uint_as_float(u0.z), __uint_as_float(u0.w),
                      __uint_as_float(u1.x), __uint_as_float(u1.y), __uint_as_float(u1.z), __uint_as_float(u1.w)};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const _Float16 hb = (_Float16)x[i];
    h[i] = hb;
    l[i] = (_Float16)(x[i] - (float)hb);
  }
}

// swizzle key of staged row r. A fragment read puts rows n = 0-3, 12-15 of k quarter q and rows 4-11 of
// quarter q ^ 1 in one ds_read_b128 lane group (MI355X_MICROARCH.md LDS table); a lane's chunks are 8c + 2q
// (+ 1), so the groups' chunks differ in bit 1: with this key (conv_halo.hip's hkey with bits 0 and 1
// swapped) the 16 chunks of ANY 16 consecutive rows differ in every group (tools/swizzle_search.py; key
// r & 15 was 2-way conflicted at every shift)
MZ_DEV int xkey(int r) { return (r & 1) | (((r >> 2) & 1) * 10) | (((r >> 1) & 1) << 2); }

template <int CIN, int TM>
__global__ __launch_bounds__(x6::NT, 1) void conv_x6_kernel(X6Args a) {
  constexpr int RB = CIN * 4;        // bytes per staged row (f32)
  constexpr int NC = RB / 16;        // 16-B chunks per row
  constexpr int NCS = CIN / 32;      // 32-channel k steps per tap
  constexpr int MT = TM / 32;        // 16-pixel tiles per wave (two pixel halves)
  static_assert(NCS % 2 == 0 && TM % 32 == 0, "ring slot = step parity; whole pixel tiles per half");
  constexpr int nsteps = 9 * NCS;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // pixel half, channel quarter (64)
  const int q = lane >> 4, n = lane & 15;
  const int m0 = blockIdx.x * TM, n0 = blockIdx.y * x6::TN;
  const int HW = a.H * a.W;

  // the zero block: 16 rows at ZOFF (16-row aligned), never overwritten by staging
  for (int i = tid; i < RB; i += x6::NT) *reinterpret_cast<uint4*>(lds + a.ZOFF + i * 16) = make_uint4(0, 0, 0, 0);

  // the lane's pixel in tile mi: staged row prow0 + 16 mi at tap (0, 0); byte mi of okw: its taps in the image
  const int prow0 = wm * (TM / 2) + n + a.HALO;
  uint32_t okw[2] = {0u, 0u};
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m0 + wm * (TM / 2) + mi * 16 + n;
    if (m < a.M) {
      const int p = m % HW, y = p / a.W, x = p - y * a.W;
      const uint32_t b = 16u | (y > 0 ? 1u : 0u) | (y < a.H - 1 ? 2u : 0u) | (x > 0 ? 4u : 0u) | (x < a.W - 1 ? 8u : 0u);
      okw[mi >> 2] |= b << (8 * (mi & 3));
    }
  }

  // weight ring: k step j = tap * NCS + channel step (the pack's own order); three parts per fragment
  const int KS = 9 * CIN / 32;
  const uint4* wbase = reinterpret_cast<const uint4*>(a.wx) + (size_t)(n0 / 16 + wn * 4) * KS * 64;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(wbase), 0, 0x7fffffff, 0x00020000);
  const int pstride = (int)(a.part * 2);  // bytes per part
  auto wload = [&](int ct, int part, int s) {
    s = s < nsteps ? s : nsteps - 1;
    return __builtin_bit_cast(bf16x8,
                              __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, part * pstride + (ct * KS + s) * 1024, 0));
  };
  bf16x8 bq[2][3][4];  // [step parity][part][column tile]
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int pt = 0; pt < 3; ++pt)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) bq[cc][pt][ct] = wload(ct, pt, cc);

  f32x4 acc[MT][4];
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[mi][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // stage rows [m0 - HALO, m0 - HALO + TM + 2 HALO) x all Cin channels (f32): 1-KiB block i holds chunks
  // 64 i .. 64 i + 63 (row g / NC, physical chunk g % NC = logical chunk ^ xkey(row))
  for (int i = wave; i < a.NI; i += 8) {
    const int g = i * 64 + lane, r = g / NC, s = g - r * NC;
    int m = m0 - a.HALO + r;
    m = m < 0 ? 0 : (m >= a.M ? a.M - 1 : m);
    const float* src = a.in + (size_t)m * CIN + ((s ^ xkey(r)) << 2);
    __builtin_amdgcn_global_load_lds(src, lds + i * 1024, 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // a tap's row offsets per pixel tile; a tap that leaves the image reads row (r & 15) of the zero block, the
  // bank slot its own row would take (one shared zero row cost 0.44 of the LDS-active cycles in bank conflicts
  // at the 4x5 latent, where 14 of 20 pixels are on the border: profiles/r04/r4f/psq2_x6.json). The row's key is
  // recomputed from the offset at each read (kept beside the offsets, the keys spilled)
  auto tap_set = [&](int t, int (&rb)[MT]) {
    const int dy = t / 3 - 1, dx = t % 3 - 1;
    const uint32_t need = 16u | (dy < 0 ? 1u : 0u) | (dy > 0 ? 2u : 0u) | (dx < 0 ? 4u : 0u) | (dx > 0 ? 8u : 0u);
    const int shift = dy * a.W + dx;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const bool ok = ((okw[mi >> 2] >> (8 * (mi & 3))) & need) == need;
      const int r = prow0 + 16 * mi + shift;
      rb[mi] = ok ? r * RB : a.ZOFF + (r & 15) * RB;
    }
  };
  // the 8 f32 channels 32 c + 8 q .. of the lane's row: chunks 8c + 2q, 8c + 2q + 1 (swizzled by xkey(row))
  auto frag = [&](const int (&rb)[MT], int c, int mi, uint4& u0, uint4& u1) {
    const int ch = 8 * c + 2 * q;
    const int key = xkey(((unsigned)rb[mi] / RB) & 15);
    u0 = *reinterpret_cast<const uint4*>(lds + rb[mi] + ((ch ^ key) << 4));
    u1 = *reinterpret_cast<const uint4*>(lds + rb[mi] + (((ch + 1) ^ key) << 4));
  };
  constexpr int NF = MT * NCS;  // fragments per tap in (channel step, pixel tile) order
  static_assert(NF % 2 == 0, "rolling buffer");

  int rbc[MT], rbn[MT];
  tap_set(0, rbc);
  // software pipeline over the flat fragment sequence (tap, channel step, pixel tile): fragment i's 24 MFMAs
  // run while fragment i + 1 is split into its bf16 parts (VALU, interleaved below) and fragment i + 2 is read
  // from LDS. Split in place just before its own MFMAs, the ~50 VALU of a split stalled the wave between
  // fragments.
  uint4 f0[2], f1[2];  // raw f32 fragments, slot = index parity (NF is even)
  bf16x8 sp[2][3];     // split parts (hi, mid, lo), slot = index parity
  frag(rbc, 0, 0, f0[0], f1[0]);
  frag(rbc, NF > 1 ? 1 / MT : 0, 1 % MT, f0[1], f1[1]);
  split8(f0[0], f1[0], sp[0][0], sp[0][1], sp[0][2]);
  int j = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    tap_set(t < 8 ? t + 1 : t, rbn);
#pragma unroll
    for (int c = 0; c < NCS; ++c) {
      const int sl = c & 1;
      const int sn = j + 2;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int idx = c * MT + mi, n1 = idx + 1, n2 = idx + 2;
        if (n2 < NF)
          frag(rbc, n2 / MT, n2 % MT, f0[n2 & 1], f1[n2 & 1]);
        else if (t < 8)
          frag(rbn, (n2 - NF) / MT, (n2 - NF) % MT, f0[n2 & 1], f1[n2 & 1]);
        if (n1 < NF || t < 8) split8(f0[n1 & 1], f1[n1 & 1], sp[n1 & 1][0], sp[n1 & 1][1], sp[n1 & 1][2]);
        const bf16x8 &xh = sp[idx & 1][0], &xm = sp[idx & 1][1], &xl = sp[idx & 1][2];
        // per accumulator the small terms first, then the large ones (each an f32-accumulating bf16 MFMA);
        // issued term-major across the column tiles, so consecutive MFMAs are independent
        const bf16x8* xs[6] = {&xh, &xm, &xl, &xh, &xm, &xh};
        constexpr int wp[6] = {2, 1, 0, 1, 0, 0};
#pragma unroll
        for (int k = 0; k < 6; ++k)
#pragma unroll
          for (int ct = 0; ct < 4; ++ct)
            acc[mi][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[sl][wp[k]][ct], *xs[k], acc[mi][ct], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // the LDS reads of fragment i + 2 first
#pragma unroll
        for (int k = 0; k < 24; ++k) {  // then each MFMA with two VALU of the next split in its shadow
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int pt = 0; pt < 3; ++pt)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) bq[sl][pt][ct] = wload(ct, pt, sn);
      __builtin_amdgcn_sched_barrier(0);
      ++j;
    }
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) rbc[mi] = rbn[mi];
  }

  // epilogue (f32): acc[mi][ct] = D[channel n0 + 64 wn + 16 ct + 4q + i][pixel m0 + TM/2 wm + 16 mi + n]
  const int nb = n0 + wn * 64;
  float4 bb[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) bb[ct] = *reinterpret_cast<const float4*>(a.bias + nb + ct * 16 + 4 * q);
  const float lo = a.relu ? 0.f : -__builtin_inff();
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m0 + wm * (TM / 2) + mi * 16 + n;
    const int mc = m < a.M ? m : a.M - 1;
    float4 rv[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
      rv[ct] = a.res ? *reinterpret_cast<const float4*>(a.res + (size_t)mc * a.Cout + nb + ct * 16 + 4 * q)
                     : make_float4(-0.f, -0.f, -0.f, -0.f);  // (acc + bias) + -0 is acc + bias
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      float4 o;
      o.x = fmaxf((acc[mi][ct][0] + bb[ct].x) + rv[ct].x, lo);
      o.y = fmaxf((acc[mi][ct][1] + bb[ct].y) + rv[ct].y, lo);
      o.z = fmaxf((acc[mi][ct][2] + bb[ct].z) + rv[ct].z, lo);
      o.w = fmaxf((acc[mi][ct][3] + bb[ct].w) + rv[ct].w, lo);
      if (m < a.M) *reinterpret_cast<float4*>(a.out + (size_t)m * a.Cout + nb + ct * 16 + 4 * q) = o;
    }
  }
}

// Pre-split form (default where it fits): the staging goes through registers and splits every f32 value ONCE
// into its hi / mid / lo bf16 parts, stored as three planes per staged row (row = hi[Cin] | mid[Cin] | lo[Cin],
// 16-B chunks XOR-swizzled by hkey(row) within each plane, conv_halo.hip's key: bf16 chunks 4c + q); the k loop
// then reads MFMA-ready operands (three ds_read_b128 per fragment, no VALU). conv_x6_kernel splits per fragment
// read, i.e. each staged value 9 taps x 4 channel-quarter waves = 36 times, and that split was 24 % of its time
// by ablation (profiles/r04/x6_abl/). The 8 waves own 32 output channels each over all TM pixels (no weight
// fragment streamed twice per workgroup); a row is 1.5x the f32 row, so TM is 80 at the 4x5 latent (1 024
// tiles at B = 4 096: four rounds of 256 CUs exactly). Same products, same order per accumulator: bit-identical
// to conv_x6_kernel.
MZ_DEV int pkey(int r) { return ((r << 1) & 6) | (((r >> 2) & 1) * 9); }  // = conv_halo.hip hkey

// CT: 16-channel column tiles per wave (2: 256 output channels per workgroup; 1: 128, the Cout 128 convs). NBLK:
// the input channels staged in NBLK blocks of CIN / NBLK (round 5: the 16x20 Cin-256 convs in two 128-channel blocks,
// so a 160-pixel tile's 1.5x rows fit — one block took 48-pixel tiles there, each streaming all 3.5 MB of weight
// parts, the L2 weight stream then bounding it); NBLK > 1 sums (block, tap, channel step) in that order.
// NP = 2 (round 6): the split-fp16 x3 form of conv_x6t (§3.6 of DESIGN.md) on these tiles — two fp16 planes per row,
// three fp16 MFMAs per product, weights scaled by 2^k per output channel (undone in the epilogue): the f32 path's
// 16x20 / 8x10 representation convs.
template <int CIN, int TM, int CT = 2, int NBLK = 1, int NP = 3>
__global__ __launch_bounds__(x6::NT, 1) void conv_x6p_kernel(X6Args a) {
  using V8 = std::conditional_t<NP == 3, bf16x8, f16x8>;
  constexpr int CB = CIN / NBLK;     // channels per staged block
  constexpr int PB = CB * 2;         // bytes per plane row (bf16 / fp16)
  constexpr int RB = NP * PB;        // bytes per staged row: hi | mid | lo (x3: hi | lo)
  constexpr int NC8 = CB / 8;        // 8-channel chunks per row
  constexpr int NCS = CB / 32;       // 32-channel k steps per tap and block
  constexpr int MT = TM / 16;        // pixel tiles per wave: all of the workgroup's
  static_assert(NCS % 2 == 0 && TM % 16 == 0 && MT <= 10, "ring slot = step parity; whole pixel tiles");
  constexpr int nsteps = NBLK * 9 * NCS;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, n = lane & 15;
  const int m0 = blockIdx.x * TM, n0 = blockIdx.y * (128 * CT);
  const int HW = a.H * a.W;
  const int HR = TM + 2 * a.HALO;

  for (int i = tid; i < RB / 16; i += x6::NT) *reinterpret_cast<uint4*>(lds + a.ZOFF + i * 16) = make_uint4(0, 0, 0, 0);

  int prow0 = n + a.HALO;
  uint32_t okw[(MT + 3) / 4] = {};
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m0 + mi * 16 + n;
    if (m < a.M) {
      const int p = m % HW, y = p / a.W, x = p - y * a.W;
      const uint32_t b = 16u | (y > 0 ? 1u : 0u) | (y < a.H - 1 ? 2u : 0u) | (x > 0 ? 4u : 0u) | (x < a.W - 1 ? 8u : 0u);
      okw[mi >> 2] |= b << (8 * (mi & 3));
    }
  }

  const int KS = 9 * CIN / 32;
  const uint4* wbase = reinterpret_cast<const uint4*>(a.wx) + (size_t)(n0 / 16 + wave * CT) * KS * 64;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(wbase), 0, 0x7fffffff, 0x00020000);
  const int pstride = (int)(a.part * 2);
  // loop step j = (block, tap, channel step) -> pack k step tap * CIN / 32 + block * NCS + c
  auto wload = [&](int ct, int part, int j) {
    j = j < nsteps ? j : nsteps - 1;
    const int blk = j / (9 * NCS), r = j - blk * 9 * NCS, t = r / NCS, c = r - t * NCS;
    const int s = t * (CIN / 32) + blk * NCS + c;
    return __builtin_bit_cast(V8,
                              __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, part * pstride + (ct * KS + s) * 1024, 0));
  };
  V8 bq[2][NP][CT];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int pt = 0; pt < NP; ++pt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) bq[cc][pt][ct] = wload(ct, pt, cc);

  f32x4 acc[MT][CT];
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[mi][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // staging of block blk: item g = (row, 8-channel chunk); 8 f32 loaded, split, written as one chunk per plane.
  // Loads of a batch of 8 items are all issued before its first split.
  const int items = HR * NC8;
  auto stage = [&](int blk) {
    for (int g0 = 0; g0 < items; g0 += 8 * x6::NT) {
      uint4 v[8][2];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int g = min(g0 + u * x6::NT + tid, items - 1), r = g / NC8, s8 = g - r * NC8;
        int m = m0 - a.HALO + r;
        m = m < 0 ? 0 : (m >= a.M ? a.M - 1 : m);
        const float* src = a.in + (size_t)m * CIN + blk * CB + s8 * 8;
        v[u][0] = *reinterpret_cast<const uint4*>(src);
        v[u][1] = *reinterpret_cast<const uint4*>(src + 4);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int g = g0 + u * x6::NT + tid;
        if (g < items) {
          const int r = g / NC8, s8 = g - r * NC8;
          uint8_t* row = lds + r * RB + ((s8 ^ pkey(r)) << 4);
          if constexpr (NP == 3) {
            bf16x8 h, mm, l;
            split8(v[u][0], v[u][1], h, mm, l);
            *reinterpret_cast<bf16x8*>(row) = h;
            *reinterpret_cast<bf16x8*>(row + PB) = mm;
            *reinterpret_cast<bf16x8*>(row + 2 * PB) = l;
          } else {
            f16x8 h, l;
            split8h(v[u][0], v[u][1], h, l);
            *reinterpret_cast<f16x8*>(row) = h;
            *reinterpret_cast<f16x8*>(row + PB) = l;
          }
        }
      }
    }
  };

  // fragment of pixel tile mi, channel step c at tap t: chunk 4c + q of the three planes of its row (the zero row
  // for a tap leaving the image; its bank slots collide with at most a few lanes', measured neutral for conv_x6)
  auto frag = [&](int t, int c, int mi, V8 (&f)[NP]) {
    const int dy = t / 3 - 1, dx = t % 3 - 1;
    const uint32_t need = 16u | (dy < 0 ? 1u : 0u) | (dy > 0 ? 2u : 0u) | (dx < 0 ? 4u : 0u) | (dx > 0 ? 8u : 0u);
    const bool ok = ((okw[mi >> 2] >> (8 * (mi & 3))) & need) == need;
    const int r = prow0 + 16 * mi + dy * a.W + dx;
    const int base = ok ? r * RB + (((4 * c + q) ^ pkey(r)) << 4) : a.ZOFF;
#pragma unroll
    for (int pt = 0; pt < NP; ++pt) f[pt] = *reinterpret_cast<const V8*>(lds + base + pt * PB);
  };
  constexpr int NF = MT * NCS;
  int j = 0;
#pragma unroll
  for (int blk = 0; blk < NBLK; ++blk) {
    if (blk > 0) __syncthreads();  // every wave is done with the previous block's rows
    if (NBLK > 1) {  // opaque per block: the fragment addresses CSE'd across the unrolled blocks spill (conv_halo.hip)
      asm volatile("" : "+v"(prow0));
#pragma unroll
      for (int i = 0; i < (MT + 3) / 4; ++i) asm volatile("" : "+v"(okw[i]));
    }
    stage(blk);
    __syncthreads();
    V8 fr[2][NP];  // rolling: fragment i + 1 read during fragment i's MFMAs
    frag(0, 0, 0, fr[0]);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
#pragma unroll
      for (int c = 0; c < NCS; ++c) {
        const int sl = c & 1;
        const int sn = j + 2;
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          const int idx = c * MT + mi, nx = idx + 1;
          // the flat fragment index parity picks the buffer: NF may be odd, so count across taps
          const int cur = (t * NF + idx) & 1, nxt = cur ^ 1;
          if (nx < NF)
            frag(t, nx / MT, nx % MT, fr[nxt]);
          else if (t < 8)
            frag(t + 1, 0, 0, fr[nxt]);
          // per accumulator the small terms first, as conv_x6_kernel: x6 (w, x) parts (2,0) (1,1) (0,2) (1,0) (0,1)
          // (0,0); x3 (1,0) (0,1) (0,0)
          constexpr int NTM = NP == 3 ? 6 : 3;
          constexpr int wp6[6] = {2, 1, 0, 1, 0, 0}, xp6[6] = {0, 1, 2, 0, 1, 0};
          constexpr int wp3[3] = {1, 0, 0}, xp3[3] = {0, 1, 0};
#pragma unroll
          for (int k = 0; k < NTM; ++k)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
              if constexpr (NP == 3)
                acc[mi][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[sl][wp6[k]][ct], fr[cur][xp6[k]], acc[mi][ct], 0, 0, 0);
              else
                acc[mi][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[sl][wp3[k]][ct], fr[cur][xp3[k]], acc[mi][ct], 0, 0, 0);
            }
          __builtin_amdgcn_sched_group_barrier(0x100, NP, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NTM * CT, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int pt = 0; pt < NP; ++pt)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) bq[sl][pt][ct] = wload(ct, pt, sn);
        __builtin_amdgcn_sched_barrier(0);
        ++j;
      }
    }
  }

  // epilogue (f32): acc[mi][ct] = D[channel n0 + 32 wave + 16 ct + 4q + i][pixel m0 + 16 mi + n]
  const int nb = n0 + wave * 16 * CT;
  float4 bb[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) bb[ct] = *reinterpret_cast<const float4*>(a.bias + nb + ct * 16 + 4 * q);
  if constexpr (NP == 2) {  // undo the weights' 2^k (exact)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const float4 sc = *reinterpret_cast<const float4*>(a.wscale + nb + ct * 16 + 4 * q);
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) acc[mi][ct] *= f32x4{sc.x, sc.y, sc.z, sc.w};
    }
  }
  const float lo = a.relu ? 0.f : -__builtin_inff();
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m0 + mi * 16 + n;
    const int mc = m < a.M ? m : a.M - 1;
    float4 rv[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      rv[ct] = a.res ? *reinterpret_cast<const float4*>(a.res + (size_t)mc * a.Cout + nb + ct * 16 + 4 * q)
                     : make_float4(-0.f, -0.f, -0.f, -0.f);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float4 o;
      o.x = fmaxf((acc[mi][ct][0] + bb[ct].x) + rv[ct].x, lo);
      o.y = fmaxf((acc[mi][ct][1] + bb[ct].y) + rv[ct].y, lo);
      o.z = fmaxf((acc[mi][ct][2] + bb[ct].z) + rv[ct].z, lo);
      o.w = fmaxf((acc[mi][ct][3] + bb[ct].w) + rv[ct].w, lo);
      if (m < a.M) *reinterpret_cast<float4*>(a.out + (size_t)m * a.Cout + nb + ct * 16 + 4 * q) = o;
    }
  }
}

// Pixel-tiled form for the 4x5 latent at full batches (round 5; conv_x6t): a workgroup owns 16 whole envs, all
// 20 pixels, and an MFMA column tile is ONE pixel of those 16 envs (towerp.hip's tiling), so a 3x3 tap maps pixel
// tile p onto pixel tile p + dy W + dx whole and the 50 of 180 tile-taps that fall on the zero padding
// (Conv2d(padding=1) on the 4x5 latent) are not issued: 0.72 of conv_x6p's MFMAs, where every 16-pixel tile
// runs all 9 taps (the zero block for the out-of-image rows). 16 envs x 20 pixels x 256 channels as three bf16
// planes are 480 KiB, so the input channels are staged in 8 blocks of 32: the next block's f32 rows come in by
// LDS-DMA (40 KiB, issued when the previous split ends) while the current block's k steps run; at a block end
// the raw rows are split once into the hi / mid / lo planes (3 x 20 KiB; row (pixel p, env e) = 16 p + e,
// 64 B per plane row, chunk q ^ key(e): any 16 rows of a tile conflict-free, tools/swizzle search). 8 waves, each
// 16 output channels x all 20 pixel tiles (acc 20, pinned to AGPRs), so a workgroup owns 128 output channels
// (grid.y = Cout / 128; 32 channels per wave need 160 accumulators beside the ring: 300 VGPRs spilled at two waves
// per SIMD, and one wave per SIMD would need 320 accumulators for all 256); weights from the 'wx' pack through
// a two-step register ring, k step j = (block b, tap t) -> pack step 8 t + b. Per accumulator the order is
// (channel block, tap, the six terms small first): the same products as conv_x6p in another order, so the two
// agree to f32 rounding (both as close to exact as an f32 conv), not bit for bit.
// GA: the input gathered per env from the latent pool (in + b env_stride + slot[b] slot_stride) and the
// action-bias table added ((acc + act_bias) + bias, conv_igemm's order): the f32 dynamics' first conv.
namespace x6t {
constexpr int E = 16, HW = 20, H = 4, W = 5, CIN = 256, NCS = 8;
constexpr int ROWS = HW * E;          // 320 staged rows (pixel, env)
constexpr int PB = ROWS * 64;         // bytes per 16-bit plane of a 32-channel block
// NP planes (3: the bf16 x6 form, 2: the fp16 x3 form), then the f32 rows of the next block: 320 x 128 B
// pipe (round 6): two plane sets, the next block's split into the idle one during the current block's k loop
constexpr int raw(int np, bool pipe = false) { return np * PB * (pipe ? 2 : 1); }
constexpr int lds(int np, bool pipe = false) { return raw(np, pipe) + ROWS * 128; }  // 100 / 80 KiB; piped 160 / 120
}  // namespace x6t

// the (tap, output pixel) pairs of a 3x3 conv on the 4x5 latent whose source pixel is in the image: 130 of 180
struct X6TPairs {
  int n = 0;
  int tap[180] = {}, out[180] = {}, src[180] = {};
  bool last[180] = {};  // the tap's last pair
};
constexpr X6TPairs make_x6t_pairs() {
  X6TPairs r{};
  for (int t = 0; t < 9; ++t) {
    const int dy = t / 3 - 1, dx = t % 3 - 1;
    for (int p = 0; p < x6t::HW; ++p) {
      const int y = p / x6t::W + dy, x = p % x6t::W + dx;
      if (y < 0 || y >= x6t::H || x < 0 || x >= x6t::W) continue;
      r.tap[r.n] = t, r.out[r.n] = p, r.src[r.n] = y * x6t::W + x;
      ++r.n;
    }
    r.last[r.n - 1] = true;
  }
  return r;
}
constexpr X6TPairs kPairs = make_x6t_pairs();
static_assert(kPairs.n == 130, "130 of the 180 tile-taps of a 4x5 latent are in the image");

// the same pairs grouped by (dy, source pixel), dy-major, sources ascending: one B fragment read feeds the group's
// 1-3 output pixels (dx = -1, 0, +1 ascending), so per accumulator the taps still come dy-major, dx ascending
struct X6TGroups {
  int n = 0;
  int dy[60] = {}, src[60] = {}, cnt[60] = {}, out[60][3] = {}, dx[60][3] = {};
  bool last[60] = {};  // the dy row's last group
  int last_first = 0;  // the first dy row's last group (the block's first ring reload)
};
// ks = 3: the 3x3 conv's groups; ks = 1: the centre tap only (a 1x1 conv: 20 groups of one pixel each)
constexpr X6TGroups make_x6t_groups(int ks) {
  X6TGroups r{};
  int pairs = 0;
  for (int dy = -1; dy <= 1; ++dy) {
    if (ks == 1 && dy != 0) continue;
    for (int ps = 0; ps < x6t::HW; ++ps) {
      const int ys = ps / x6t::W, xs = ps % x6t::W, y = ys - dy;
      if (y < 0 || y >= x6t::H) continue;
      int c = 0;
      for (int dx = -1; dx <= 1; ++dx) {
        if (ks == 1 && dx != 0) continue;
        const int x = xs - dx;
        if (x < 0 || x >= x6t::W) continue;
        r.out[r.n][c] = y * x6t::W + x, r.dx[r.n][c] = dx + 1;
        ++c;
      }
      r.dy[r.n] = ks == 3 ? dy + 1 : 0, r.src[r.n] = ps, r.cnt[r.n] = c;  // dy: the ring step within a block
      pairs += c;
      ++r.n;
    }
    r.last[r.n - 1] = true;
  }
  r.n = pairs == (ks == 3 ? 130 : 20) ? r.n : -1;
  for (int i = 0; i < 60; ++i)
    if (r.last[i]) {
      r.last_first = i;
      break;
    }
  return r;
}
constexpr X6TGroups kGroups = make_x6t_groups(3);
constexpr X6TGroups kGroups1 = make_x6t_groups(1);

// f(std::integral_constant<int, i>) for i = 0 .. N - 1, each a compile-time index (the group tables index
// sched_group_barrier counts, which must be constants)
template <typename F, size_t... Is>
MZ_DEV void x6t_static_for_impl(F&& f, std::index_sequence<Is...>) {
  (f(std::integral_constant<int, (int)Is>()), ...);
}
template <int N, typename F>
MZ_DEV void x6t_static_for(F&& f) {
  x6t_static_for_impl(f, std::make_index_sequence<N>());
}
static_assert(kGroups.n == 50, "15 + 20 + 15 source pixels, 130 (tap, pixel) pairs");
static_assert(kGroups1.n == 20, "a 1x1 conv: 20 (centre tap, pixel) pairs");

struct X6TArgs {
  const float* in;
  long long env_stride;   // elements between envs (contiguous: 20 x 256)
  const int32_t* slot;    // optional: env b's image at in + b env_stride + slot[b] slot_stride
  long long slot_stride;
  const bf16_t* wx;       // [3 parts][Cout / 16][9 or 1 taps x 8][64][8]
  const float* bias;      // [Cout]
  const float* act_bias;  // optional [20][A][Cout] (GA)
  const int32_t* act;     // [B] (GA)
  int A;
  const float* res;       // optional [B][20][Cout]
  float* out;             // [B][20][Cout]
  int B, Cout, relu;
  long long part;         // elements per weight part
  const float* wscale;    // x3 form: per output channel, 2^-k of the host's weight scaling (exact); x6: unused
};

MZ_DEV int tkey(int e) { return (e >> 2) & 2; }  // chunk swizzle of row 16 p + e (64-B plane rows)

// NW waves of 16 output channels each: 8 (128 channels per workgroup, the default) or 4 (64 channels: twice the
// workgroups where the 8-wave grid leaves CUs idle, config 2's 1 024 envs; per wave the same arithmetic)
#ifndef X3_ABLATE
#define X3_ABLATE 0  // diagnostic builds only (numerically wrong): 1 no per-block staging / split, 2 no ring reloads
#endif
#ifndef X3_ASM_RING
#define X3_ASM_RING 0  // A/B build (-DX3_ASM_RING=1): the pipelined x3 form's ring loads, DMA and raw reads as inline asm with explicit waits (+0.6 %)
#endif
#ifndef X3_PFD
#define X3_PFD 2  // the x3 form's fragment prefetch distance in (dy, source pixel) groups (A/B: -DX3_PFD=1)
#endif

// s_waitcnt vmcnt(N) for the ring depths below
template <int N>
MZ_DEV void x6t_wait_vm() {
  static_assert(N == 27 || N == 18 || N == 12 || N == 3 || N == 2 || N == 0, "ring wait depth");
  if constexpr (N == 27)
    asm volatile("s_waitcnt vmcnt(27)" ::: "memory");
  else if constexpr (N == 0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 18)
    asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else if constexpr (N == 12)
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 3)
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
}

// NP = 3: the bf16 x6 form above. NP = 2 (round 6): split-fp16 x3 — x = xh + xl (fp16 hi / lo, split8h), the weights
// likewise from w 2^k (k per output channel, so every weight's lo part stays normal: agent.py split_pack_x3), and a
// product as the three terms xh wl + xl wh + xh wh (xl wl, below 2^-22 of the product, dropped) on
// v_mfma_f32_16x16x32_f16, f32 accumulate; the accumulator times 2^-k in the epilogue (exact). About 22 significant
// bits per operand at half the MFMAs of x6 (tests/test_gpu_parity.py: the nets at 1e-5 of the reference)
//
// PIPE (round 6): no split phase between the blocks. Each wave splits only the raw rows its own LDS-DMA pieces
// brought in (so its own vmcnt is the only wait: no barrier between the DMA and the split), into the idle one of
// two plane sets, in a few sub-steps between the first (dy, source pixel) groups of the block before, then re-issues
// its DMA pieces for the block after into the same rows; one barrier per block publishes the new planes. Same
// products in the same order: bit-identical to PIPE = false.
template <bool GA, int KSZ = 3, int NW = 8, int NP = 3, bool PIPE = false>
// (the 4-wave x3 form without PIPE: 80 KiB of LDS and at most 256 registers a lane, so two workgroups share a CU and
// one's split phase and barriers overlap the other's k loop — mzba_conv_x3_set_pipe(2))
__global__ __launch_bounds__(64 * NW, (NW == 4 && NP == 2 && !PIPE) ? 2 : 1) void conv_x6t_kernel(X6TArgs a) {
  using namespace x6t;
  static_assert(NP == 3 || NP == 2, "x6 (bf16) or x3 (fp16)");
  using V8 = std::conditional_t<NP == 3, bf16x8, f16x8>;
  constexpr int RAW = raw(NP, PIPE);
  constexpr int NT = 64 * NW;
  constexpr const X6TGroups& G = KSZ == 3 ? kGroups : kGroups1;
  constexpr int SPB = KSZ == 3 ? 3 : 1;     // ring steps per channel block (the dy rows)
  constexpr int KST = KSZ * KSZ * NCS;      // pack k steps per column tile
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, n = lane & 15;
  const int e0 = blockIdx.x * E;
  const int nb = blockIdx.y * (16 * NW) + wave * 16;  // the wave's first output channel

  // LDS-DMA of block cb's f32 rows: 1-KiB piece i = rows 8 i .. 8 i + 7 = pixel i >> 1, envs 8 (i & 1) + 0..7; the
  // waves take pieces wave + NW k (NW even), so a lane's env (8 (wave & 1) + lane / 8) is fixed: its offset is read once
  const int se = min(e0 + 8 * (wave & 1) + (lane >> 3), a.B - 1);
  long long eoff = (long long)se * a.env_stride;
  if (GA && a.slot) eoff += (long long)a.slot[se] * a.slot_stride;
  const float* src0 = a.in + eoff + (lane & 7) * 4;
  // PIPE (asm ring): the DMA as inline asm too, so every vmcnt wait of the k loop is this kernel's own (a compiler-
  // tracked DMA made the compiler drain vmcnt — the ring loads just issued included — before each raw-row read)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds;
  auto stage = [&](int cb) {
#pragma unroll
    for (int k = 0; k < 40 / NW; ++k) {
      const int i = wave + NW * k;
      if constexpr (PIPE && X3_ASM_RING) {
        const float* g = src0 + (size_t)(i >> 1) * CIN + cb * 32;
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds0 + RAW + i * 1024);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0v) : "memory", "m0");
      } else {
        __builtin_amdgcn_global_load_lds(src0 + (size_t)(i >> 1) * CIN + cb * 32, lds + RAW + i * 1024, 16, 0, 0);
      }
    }
  };
  // one (row, 8-channel chunk) of the raw block into the planes at pdst
  auto split_item = [&](int r, int k8, int pdst) {
    const uint4 u0 = *reinterpret_cast<const uint4*>(lds + RAW + r * 128 + k8 * 32);
    const uint4 u1 = *reinterpret_cast<const uint4*>(lds + RAW + r * 128 + k8 * 32 + 16);
    uint8_t* row = lds + pdst + r * 64 + ((k8 ^ tkey(r & 15)) << 4);
    if constexpr (NP == 3) {
      bf16x8 h, m, l;
      split8(u0, u1, h, m, l);
      *reinterpret_cast<bf16x8*>(row) = h;
      *reinterpret_cast<bf16x8*>(row + PB) = m;
      *reinterpret_cast<bf16x8*>(row + 2 * PB) = l;
    } else {
      f16x8 h, l;
      split8h(u0, u1, h, l);
      *reinterpret_cast<f16x8*>(row) = h;
      *reinterpret_cast<f16x8*>(row + PB) = l;
    }
  };
  // PIPE: sub-step u of this wave's own rows (its DMA pieces wave + NW k, 8 rows x 4 chunks each): item lane + 64 u
  constexpr int PPW = 40 / NW, NSUB = (PPW + 1) / 2;
  auto split_own = [&](int u, int pdst) {
    const int idx = lane + 64 * u, k = idx >> 5;
    if (k < PPW) split_item(8 * (wave + NW * k) + ((idx & 31) >> 2), idx & 3, pdst);
  };
  // the same in two halves (the reads one group ahead of the conversion); lanes past the wave's last piece redo the
  // last one (the same values to the same addresses), so no lane branches
  auto own_row = [&](int u, int& r, int& k8) {
    const int idx = lane + 64 * u, k = min(idx >> 5, PPW - 1);
    r = 8 * (wave + NW * k) + ((idx & 31) >> 2), k8 = idx & 3;
  };
  auto raw_read = [&](int u, u32x4 (&v)[2]) {
    int r, k8;
    own_row(u, r, k8);
    if constexpr (PIPE && X3_ASM_RING) {  // untracked like the DMA (the compiler would drain vmcnt before it)
      const uint32_t ad = lds0 + RAW + r * 128 + k8 * 32;
      u32x4 a0, a1;
      asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16" : "=&v"(a0), "=&v"(a1) : "v"(ad) : "memory");
      v[0] = a0, v[1] = a1;
    } else {
      v[0] = *reinterpret_cast<const u32x4*>(lds + RAW + r * 128 + k8 * 32);
      v[1] = *reinterpret_cast<const u32x4*>(lds + RAW + r * 128 + k8 * 32 + 16);
    }
  };
  auto raw_split_write = [&](int u, const u32x4 (&vv)[2], int pdst) {
    int r, k8;
    own_row(u, r, k8);
    const uint4 v[2] = {__builtin_bit_cast(uint4, vv[0]), __builtin_bit_cast(uint4, vv[1])};
    uint8_t* row = lds + pdst + r * 64 + ((k8 ^ tkey(r & 15)) << 4);
    if constexpr (NP == 3) {
      bf16x8 h, m, l;
      split8(v[0], v[1], h, m, l);
      *reinterpret_cast<bf16x8*>(row) = h;
      *reinterpret_cast<bf16x8*>(row + PB) = m;
      *reinterpret_cast<bf16x8*>(row + 2 * PB) = l;
    } else {
      f16x8 h, l;
      split8h(v[0], v[1], h, l);
      *reinterpret_cast<f16x8*>(row) = h;
      *reinterpret_cast<f16x8*>(row + PB) = l;
    }
  };
  // split of the raw block into the three planes: item g = (row, 8-channel chunk)
  auto split = [&]() {
#pragma unroll
    for (int u = 0; u < (ROWS * 4 + NT - 1) / NT; ++u) {
      const int g = tid + u * NT;
      if (g < ROWS * 4) {
        const int r = g >> 2, k8 = g & 3;
        const uint4 u0 = *reinterpret_cast<const uint4*>(lds + RAW + r * 128 + k8 * 32);
        const uint4 u1 = *reinterpret_cast<const uint4*>(lds + RAW + r * 128 + k8 * 32 + 16);
        uint8_t* row = lds + r * 64 + ((k8 ^ tkey(r & 15)) << 4);
        if constexpr (NP == 3) {
          bf16x8 h, m, l;
          split8(u0, u1, h, m, l);
          *reinterpret_cast<bf16x8*>(row) = h;
          *reinterpret_cast<bf16x8*>(row + PB) = m;
          *reinterpret_cast<bf16x8*>(row + 2 * PB) = l;
        } else {
          f16x8 h, l;
          split8h(u0, u1, h, l);
          *reinterpret_cast<f16x8*>(row) = h;
          *reinterpret_cast<f16x8*>(row + PB) = l;
        }
      }
    }
  };

  // weight ring: step j = 3 b + d (block b, dy = d - 1) holds the three dx taps t = 3 d + i (pack step 8 t + b) x
  // the three parts; slot j & 1. A 1x1 conv: step j = b, the centre tap only (pack step b).
  const uint4* wbase = reinterpret_cast<const uint4*>(a.wx) + (size_t)(nb / 16) * KST * 64;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(wbase), 0, 0x7fffffff, 0x00020000);
  const int pstride = (int)(a.part * 2);
  auto wload = [&](int ti, int part, int j) {
    j = j < SPB * NCS ? j : SPB * NCS - 1;
    const int s = KSZ == 3 ? (3 * (j % 3) + ti) * 8 + j / 3 : j;
    if constexpr (PIPE && X3_ASM_RING) {
      // PIPE: the ring's loads are invisible to the compiler's wait insertion (inline asm) and waited for explicitly
      // (ring_wait): the LDS-DMA pending beside them made it wait vmcnt(0) at a row start, right after a reload
      V8 r;
      asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(r) : "v"(lane * 16), "s"(wrs),
                   "s"(part * pstride + s * 1024));
      return r;
    } else {
      return __builtin_bit_cast(V8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, part * pstride + s * 1024, 0));
    }
  };
  constexpr int T0 = KSZ == 3 ? 0 : 1, T1 = KSZ == 3 ? 3 : 2;  // the dx taps the ring holds
  // ring loads a reload issues; after the LDS-DMA of the next block a 3x3 block issues three reloads, a 1x1 block one,
  // so waiting down to the youngest two (3x3) or one (1x1) reloads has the DMA complete
  constexpr int RL = (T1 - T0) * NP, VM = KSZ == 3 ? 2 * RL : RL;
  V8 bq[2][3][NP];  // [step parity][dx tap][part]
  // PIPE (asm ring): wait until ring slot slw's loads have landed, given N vector-memory ops issued after them; the
  // slot's registers pass through each wait, so no MFMA reading them can be scheduled above it
  auto ring_wait = [&](auto nc, auto slc) __attribute__((always_inline)) {
    constexpr int N = decltype(nc)::value, SLW = decltype(slc)::value;
    static_assert(N >= 0 && N < 64, "vmcnt range");
#pragma unroll
    for (int ti = T0; ti < T1; ++ti)
#pragma unroll
      for (int pt = 0; pt < NP; ++pt) {
        V8 t = bq[SLW][ti][pt];
        asm volatile("s_waitcnt vmcnt(%1)" : "+v"(t) : "n"(N));
        bq[SLW][ti][pt] = t;
      }
  };
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int ti = T0; ti < T1; ++ti)
#pragma unroll
      for (int pt = 0; pt < NP; ++pt) bq[cc][ti][pt] = wload(ti, pt, cc);

  f32x4 acc[HW];
#pragma unroll
  for (int p = 0; p < HW; ++p) {
    acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("" : "+a"(acc[p]));
  }

  stage(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (PIPE) {  // own rows only: no barrier before the split
#pragma unroll
    for (int u = 0; u < NSUB; ++u) split_own(u, 0);
  } else {
    __syncthreads();
    split();
  }
  __syncthreads();
  stage(1);

  // the lane's B fragment of source pixel ps: row 16 ps + n, chunk q of each plane (PIPE: plane set ps0)
  const int lrow = n * 64 + ((q ^ tkey(n)) << 4);
  auto frag = [&](int ps, V8 (&f)[NP], int pset) {
#pragma unroll
    for (int pt = 0; pt < NP; ++pt) f[pt] = *reinterpret_cast<const V8*>(lds + pset + pt * PB + ps * 1024 + lrow);
  };

  // one 32-channel block: the (dy, source pixel) groups (x6t::kGroups), the next group's fragment read during the
  // current group's MFMAs; after a dy row's last group its ring slot is reloaded (step j + 2).
  // PIPE: groups 1, 3, .. (NSUB sub-steps) split block b + 1's own rows into the other plane set, after waiting for
  // the DMA the block before issued (FIRST: the prologue's, nothing younger; else the block before's SPB ring reloads
  // are younger), and group 2 NSUB re-issues the DMA for block b + 2
  auto block = [&](int b, auto par, auto first, auto bconst) __attribute__((always_inline)) {
    constexpr int P0 = decltype(par)::value;  // ring slot parity of the block's first step (SPB b) = plane set
    constexpr bool FIRST = decltype(first)::value;
    constexpr int PSET = PIPE ? P0 * NP * PB : 0, PNEXT = PIPE ? (P0 ^ 1) * NP * PB : 0;
    const bool has_next = b + 1 < NCS, has_next2 = b + 2 < NCS;

    // fragment reads PFD groups ahead: an x3 group is 6-9 MFMAs (96-144 cycles), too short to cover an LDS read
    constexpr int PFD = NP == 2 ? X3_PFD : 1;
    V8 fr[PFD + 1][NP];
#pragma unroll
    for (int j = 0; j < PFD; ++j) frag(G.src[j], fr[j], PSET);
    u32x4 rv[2];  // PIPE: the raw f32 chunk of the split item in flight
    x6t_static_for<G.n>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int d = G.dy[i], sl = (P0 + d) & 1, cur = i % (PFD + 1), cnt = G.cnt[i];
      // PIPE: block b + 1's own rows split in NSUB items, item u's raw reads in group 2u + 1 and its conversion +
      // plane writes in group 2u + 2 (interleaved with that group's MFMAs); block b + 2's DMA in group 2 NSUB + 1
      constexpr bool SPLIT = PIPE && !(X3_ABLATE & 1);
      constexpr bool RD = SPLIT && i % 2 == 1 && i / 2 < NSUB;
      constexpr bool CV = SPLIT && i >= 2 && i % 2 == 0 && i / 2 - 1 < NSUB;
      static_assert(!SPLIT || (2 * NSUB + 1 < G.last_first && G.n > 2 * NSUB + 1), "split before the first reload");
      if constexpr (PIPE && X3_ASM_RING) {  // a row's first group: its ring slot complete (counts: DESIGN §3.6)
        constexpr int BC = decltype(bconst)::value;
        constexpr int DMA = BC + 2 < NCS ? PPW : 0;  // this block's DMA for block b + 2 (issued in group 2 NSUB + 1)
        using SL = std::integral_constant<int, sl>;
        if constexpr (KSZ == 3 && i == 0) ring_wait(std::integral_constant<int, RL>(), SL());
        if constexpr (KSZ == 3 && i == G.last_first + 1) ring_wait(std::integral_constant<int, RL + DMA>(), SL());
        // (the last block issues no reloads past the last step: nothing younger than its row-0 reload, and in a
        // 1x1 conv nothing younger than the block before's)
        if constexpr (KSZ == 3 && i > G.last_first + 1 && G.last[i - 1])
          ring_wait(std::integral_constant<int, BC + 1 < NCS ? RL : 0>(), SL());
        if constexpr (KSZ == 1 && i == 0)
          ring_wait(std::integral_constant<int, BC + 1 < NCS ? RL + PPW : 0>(), SL());
      }
      if constexpr (RD) {
        if (has_next) {
          if constexpr (i == 1) x6t_wait_vm<FIRST ? 0 : SPB * RL>();
          raw_read(i / 2, rv);
        }
      }
      if constexpr (CV && !(PIPE && X3_ASM_RING)) {
        if (has_next) raw_split_write(i / 2 - 1, rv, PNEXT);
      }
      if constexpr (CV && PIPE && X3_ASM_RING) {
        if (has_next) {
          if constexpr (PIPE && X3_ASM_RING) {  // the raw reads (asm, group i - 1) landed: 2 LDS reads are younger
            u32x4 r0 = rv[0], r1 = rv[1];
            asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(r0), "+v"(r1));
            rv[0] = r0, rv[1] = r1;
          }
          raw_split_write(i / 2 - 1, rv, PNEXT);
        }
      }
      if (i + PFD < G.n) frag(G.src[i + PFD], fr[(i + PFD) % (PFD + 1)], PSET);
      // per accumulator the small terms first (conv_x6p's order): x6 (w, x) parts (2,0) (1,1) (0,2) (1,0) (0,1)
      // (0,0); x3 (1,0) (0,1) (0,0)
      constexpr int NTM = NP == 3 ? 6 : 3;
      constexpr int wp6[6] = {2, 1, 0, 1, 0, 0}, xp6[6] = {0, 1, 2, 0, 1, 0};
      constexpr int wp3[3] = {1, 0, 0}, xp3[3] = {0, 1, 0};
#pragma unroll
      for (int k = 0; k < NTM; ++k)
#pragma unroll
        for (int o = 0; o < cnt; ++o) {
          if constexpr (NP == 3)
            acc[G.out[i][o]] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[sl][G.dx[i][o]][wp6[k]], fr[cur][xp6[k]],
                                                                       acc[G.out[i][o]], 0, 0, 0);
          else
            acc[G.out[i][o]] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[sl][G.dx[i][o]][wp3[k]], fr[cur][xp3[k]],
                                                                      acc[G.out[i][o]], 0, 0, 0);
        }
      if constexpr (CV) {  // one MFMA, then up to 6 VALU of the split, ..., then the plane writes
        __builtin_amdgcn_sched_group_barrier(0x100, NP + (RD ? 2 : 0), 0);
        x6t_static_for<NTM * cnt>([&](auto) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
        });
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x100, NP + (RD ? 2 : 0), 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NTM * cnt, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      // (PIPE asm ring: no reload past the last step — an untracked load whose value is dead would land in a
      // register the compiler has meanwhile given to something else)
      if (G.last[i] && !(PIPE && (X3_ABLATE & 2)) && !(PIPE && X3_ASM_RING && SPB * b + d + 2 >= SPB * NCS)) {
#pragma unroll
        for (int ti = T0; ti < T1; ++ti)
#pragma unroll
          for (int pt = 0; pt < NP; ++pt) bq[sl][ti][pt] = wload(ti, pt, SPB * b + d + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (SPLIT && i == 2 * NSUB + 1) {
        if (has_next2) stage(b + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  };

  if constexpr (PIPE) {
    // all NCS blocks unrolled: straight-line code, so the compiler's vmcnt waits for the ring count exactly (a
    // loop back edge merged the ring's and the DMA's pending loads into vmcnt(0) waits at every block start)
    x6t_static_for<NCS>([&](auto B) {
      constexpr int b = decltype(B)::value;
      block(b, std::integral_constant<int, b & 1>(), std::integral_constant<bool, b == 0>(),
            std::integral_constant<int, b>());
      // publish the new planes: this wave's plane writes done, then the barrier alone (a __syncthreads() fence
      // drained vmcnt too — the ring loads and the DMA just issued — at every block end)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing untracked in flight into the epilogue
  } else
  for (int b = 0; b < NCS; b += 2) {
    block(b, std::integral_constant<int, 0>(), std::false_type(), std::integral_constant<int, 0>());  // SPB b even
    // block b + 1's raw rows: wait for this wave's LDS-DMA, then every wave's, then split. The DMA is older than
    // every ring load block b issued after it (VM above: a 1x1 block's one reload only — ADVICE r5)
    x6t_wait_vm<VM>();
    __syncthreads();
    split();
    __syncthreads();
    if (b + 2 < NCS) stage(b + 2);
    block(b + 1, std::integral_constant<int, 1>(), std::false_type(), std::integral_constant<int, 0>());  // SPB odd
    if (b + 2 < NCS) {
      x6t_wait_vm<VM>();
      __syncthreads();
      split();
      __syncthreads();
      if (b + 3 < NCS) stage(b + 3);
    }
  }

  // epilogue (f32): acc[p] = D[channel nb + 4 q + i][env e0 + n at pixel p]
  const int env = e0 + n;
  if (env >= a.B) return;
  const float lo = a.relu ? 0.f : -__builtin_inff();
  const int ch = nb + 4 * q;
  const float4 bb = *reinterpret_cast<const float4*>(a.bias + ch);
  if constexpr (NP == 2) {  // undo the weights' 2^k (exact)
    const float4 sc = *reinterpret_cast<const float4*>(a.wscale + ch);
#pragma unroll
    for (int p = 0; p < HW; ++p) acc[p] *= f32x4{sc.x, sc.y, sc.z, sc.w};
  }
  const int act = GA && a.act_bias ? a.act[env] : 0;
  const size_t ob = (size_t)env * HW * a.Cout;
  float4 rv[HW];
#pragma unroll
  for (int p = 0; p < HW; ++p)  // every residual / action-bias load before the first use
    rv[p] = GA && a.act_bias ? *reinterpret_cast<const float4*>(a.act_bias + ((size_t)p * a.A + act) * a.Cout + ch)
          : a.res            ? *reinterpret_cast<const float4*>(a.res + ob + (size_t)p * a.Cout + ch)
                             : make_float4(-0.f, -0.f, -0.f, -0.f);  // (acc + bias) + -0 is acc + bias
#pragma unroll
  for (int p = 0; p < HW; ++p) {
    float4 o;
    if (GA && a.act_bias) {  // (acc + act_bias) + bias
      o.x = fmaxf((acc[p][0] + rv[p].x) + bb.x, lo);
      o.y = fmaxf((acc[p][1] + rv[p].y) + bb.y, lo);
      o.z = fmaxf((acc[p][2] + rv[p].z) + bb.z, lo);
      o.w = fmaxf((acc[p][3] + rv[p].w) + bb.w, lo);
    } else {  // (acc + bias) + res
      o.x = fmaxf((acc[p][0] + bb.x) + rv[p].x, lo);
      o.y = fmaxf((acc[p][1] + bb.y) + rv[p].y, lo);
      o.z = fmaxf((acc[p][2] + bb.z) + rv[p].z, lo);
      o.w = fmaxf((acc[p][3] + bb.w) + rv[p].w, lo);
    }
    *reinterpret_cast<float4*>(a.out + ob + (size_t)p * a.Cout + ch) = o;
  }
}

// A/B: 0 conv_x6_kernel only, 1 + the pre-split form where it fits, 2 (default) + the pixel-tiled form where it
// loads the busiest CU less than the pre-split one, 3 the pixel-tiled form wherever it applies
static int g_x6_variant = 2;
// conv_x6t workgroup width: 0 auto (4 waves where the 8-wave grid leaves CUs idle), 8 or 4 forced
static int g_x6t_waves = 0;

int x6p_ncu() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  return ncu;
}

// pre-split geometry for (W, Cin, Cout, M pixels): a tile TM, the staged channel blocks NBLK and the 16-channel column
// tiles per wave CT (Cout = 128 CT per workgroup). Among the candidates whose 1.5x rows fit the LDS, the one whose
// busiest CU finishes first: rounds x max(its MFMA time, its weight stream: every tile streams all three weight parts
// of its 128 CT channels from L2 at ~67 GB/s per CU, profiles/l2_stream.json), x 1.05 for a second staging. One
// block and CT 2 everywhere up to round 4; at W >= 16 (the 16x20 representation convs: 2 (W + 1) halo rows per tile)
// also TM 160 in two 128-channel blocks (Cin 256) or one (Cin 128), and Cout 128 (CT 1). 0 if nothing fits.
struct X6PGeo {
  int tm = 0, nblk = 1, ct = 2;
};
X6PGeo x6p_geometry(int W, int Cin, int Cout, long long M, X6Args& g) {
  X6PGeo best{};
  if ((Cin != 128 && Cin != 256) || (Cout % 256 != 0 && !(Cout == 128 && Cin == 128 && W >= 16))) return best;
  double best_cost = 0;
  const int ct = Cout % 256 == 0 ? 2 : 1;
  const long long ncu = x6p_ncu();
  auto consider = [&](int tm, int nblk) {
    const int halo = W + 1, hr = tm + 2 * halo, rb = 3 * (Cin / nblk) * 2;
    if ((long long)(hr + 1) * rb > x6::LDS_MAX) return;
    const long long rounds = ((M + tm - 1) / tm * (Cout / (128 * ct)) + ncu - 1) / ncu;
    const double mfma_ns = tm * 9.0 * Cin * 128 * ct * 2 * 6 / 9.77e3;  // 2.5 PF / 256 CUs, ns
    const double wgt_ns = 3.0 * 128 * ct * 9 * Cin * 2 / 66.7;
    const double cost = rounds * (mfma_ns > wgt_ns ? mfma_ns : wgt_ns) * (nblk > 1 ? 1.05 : 1.0);
    if (!best.tm || cost < best_cost) best.tm = tm, best.nblk = nblk, best.ct = ct, best_cost = cost;
  };
  if (ct == 2)
    for (int tm : {128, 112, 96, 80, 64, 48}) consider(tm, 1);
  if (W >= 16) consider(160, Cin == 256 ? 2 : 1);
  if (!best.tm) return best;
  g.HALO = W + 1, g.NI = 0, g.ZOFF = (best.tm + 2 * (W + 1)) * 3 * (Cin / best.nblk) * 2;
  return best;
}

// the pixel tile for (W, Cin): 96, or 64 when that halo does not fit the LDS; 0 if neither fits
int x6_geometry(int W, int Cin, X6Args& g) {
  if (Cin != 128 && Cin != 256) return 0;
  for (int tm : {96, 64}) {  // 128: the ring, 64 accumulators and the split fragments spill
    const int halo = W + 1, hr = tm + 2 * halo, rb = Cin * 4;
    const int ni = (hr * rb + 1023) / 1024, zoff = (ni * 1024 + 16 * rb - 1) / (16 * rb) * (16 * rb);
    if (zoff + 16 * rb <= x6::LDS_MAX) {
      g.HALO = halo, g.NI = ni, g.ZOFF = zoff;
      return tm;
    }
  }
  return 0;
}

int x6_halo_launch(const void* in, const void* wx, const float* bias, const void* res, void* out, int B, int H, int W,
                   int Cin, int Cout, int relu, hipStream_t stream);
int x3_halo_launch(const void* in, const void* wx3, const float* wscale, const float* bias, const void* res, void* out,
                   int B, int H, int W, int Cin, int Cout, int relu, hipStream_t stream, bool dry = false);

// conv_x6t_kernel's grid for t.B envs: 4-wave (64-channel) workgroups where the 8-wave grid leaves CUs idle
// (mzba_conv_x6_set_waves: auto / 8 / 4)
template <int NP, bool PIPE>
void x6t_launch(const X6TArgs& t, int ks, bool ga, hipStream_t stream, int force_nw = 0) {
  const long long t16 = (t.B + x6t::E - 1) / x6t::E;
  const int nw = force_nw ? force_nw : g_x6t_waves ? g_x6t_waves : (t16 * (t.Cout / 128) < x6p_ncu() ? 4 : 8);
  const dim3 grid((unsigned)t16, (unsigned)(t.Cout / (16 * nw)));
  auto launch = [&](auto kern, int nthreads) {
    mz_set_lds_max_once(reinterpret_cast<const void*>(kern), x6::LDS_MAX);
    hipLaunchKernelGGL(kern, grid, dim3(nthreads), x6t::lds(NP, PIPE), stream, t);
  };
  if (nw == 4) {
    if (ks == 1)
      launch(conv_x6t_kernel<false, 1, 4, NP, PIPE>, 256);
    else
      ga ? launch(conv_x6t_kernel<true, 3, 4, NP, PIPE>, 256) : launch(conv_x6t_kernel<false, 3, 4, NP, PIPE>, 256);
  } else {
    if (ks == 1)
      launch(conv_x6t_kernel<false, 1, 8, NP, PIPE>, 512);  // the reward / value heads' 1x1 ConvBlocks (never gathered)
    else
      ga ? launch(conv_x6t_kernel<true, 3, 8, NP, PIPE>, 512) : launch(conv_x6t_kernel<false, 3, 8, NP, PIPE>, 512);
  }
}
// x3 form: 1 (default) the pipelined split (PIPE), 0 the split phase between blocks (A/B; bit-identical)
static int g_x3_pipe = 1;

}  // namespace

extern "C" {

int mzba_conv_x6_supported(int H, int W, int Cin, int Cout, int ks) {
  X6Args g{};
  if ((ks == 3 || ks == 1) && H == x6t::H && W == x6t::W && Cin == x6t::CIN && (Cout == 256 || Cout == 128))
    return 1;  // conv_x6t (the 4x5 latent; 3x3 and 1x1)
  if (ks == 3 && H >= 2 && Cout == 128 && Cin == 128 && W >= 16)
    return x6p_geometry(W, Cin, Cout, (long long)H * W, g).tm > 0 ? 1 : 0;  // the pre-split form's CT 1 instance
  return ks == 3 && H >= 2 && W >= 2 && Cout % 256 == 0 && x6_geometry(W, Cin, g) > 0 ? 1 : 0;
}

// gather = 1: a slot-gathered / strided input and / or an action-bias table (conv_x6t's GA instance: the 4x5
// latent, Cin 256, Cout 256 / 128)
int mzba_conv_x6_ex_supported(int H, int W, int Cin, int Cout, int ks, int gather) {
  if (ks == 1 && gather) return 0;  // the 1x1 instance reads contiguous images only (no slot, no action bias)
  if ((ks == 3 || ks == 1) && H == x6t::H && W == x6t::W && Cin == x6t::CIN && (Cout == 256 || Cout == 128)) return 1;
  return gather ? 0 : mzba_conv_x6_supported(H, W, Cin, Cout, ks);
}

int mzba_conv_x6_ex(const void* in, long long env_stride, const int32_t* slot, long long slot_stride, const void* wx,
                    const float* bias, const float* act_bias, const int32_t* act, int A, const void* res, void* out,
                    int B, int H, int W, int Cin, int Cout, int ks, int relu, hipStream_t stream) {
  MZ_CHECK_ARG(in && wx && bias && out && B > 0, -1);
  MZ_CHECK_ARG(!act_bias || (act && A > 0 && !res), -1);
  const bool ga = slot || act_bias || env_stride != (long long)H * W * Cin;
  MZ_CHECK_ARG(mzba_conv_x6_ex_supported(H, W, Cin, Cout, ks, ga ? 1 : 0), -2);
  const long long M = (long long)B * H * W;
  MZ_CHECK_ARG(M + 256 < (1LL << 31), -3);
  bool tiled = H == x6t::H && W == x6t::W && Cin == x6t::CIN && (Cout == 256 || Cout == 128);
  if (tiled && ks == 3 && !ga && Cout % 256 == 0 && g_x6_variant < 3) {
    // the pixel tiles where they load the busiest CU less (pixel-taps issued per CU) than conv_x6p's tiles
    X6Args ap{};
    const int tmp = g_x6_variant >= 1 ? x6p_geometry(W, Cin, Cout, M, ap).tm : 0;
    const long long ncu = x6p_ncu(), t16 = (B + x6t::E - 1) / x6t::E;
    const int nwt = g_x6t_waves ? g_x6t_waves : (t16 * 2 < ncu ? 4 : 8);  // as the launch below picks
    const long long load_t = ((256 / (16 * nwt)) * t16 + ncu - 1) / ncu * x6t::E * kPairs.n * nwt / 16;
    const long long load_p = tmp ? ((M + tmp - 1) / tmp + ncu - 1) / ncu * tmp * 9 : load_t + 1;
    tiled = g_x6_variant == 2 && load_t < load_p;
  }
  if (tiled) {
    X6TArgs t{(const float*)in, env_stride, slot, slot_stride, (const bf16_t*)wx, bias, act_bias, act, A,
              (const float*)res, (float*)out, B, Cout, relu, (long long)Cout * ks * ks * Cin, nullptr};
    x6t_launch<3, false>(t, ks, ga, stream);
    MZ_LAUNCH_CHECK();
    return 0;
  }
  return x6_halo_launch(in, wx, bias, res, out, B, H, W, Cin, Cout, relu, stream);
}

// the split-fp16 x3 form of the pixel-tiled conv (conv_x6t_kernel<.., NP = 2>): the 4x5 latent, Cin 256, Cout 256 /
// 128, 3x3 (gathered / action-biased like conv_x6_ex) or 1x1 (contiguous). wx3 = the two fp16 parts of w 2^k in the
// pack_lat16 packing back to back (agent.py split_pack_x3), wscale[Cout] = 2^-k.
int mzba_conv_x3_supported(int H, int W, int Cin, int Cout, int ks, int gather) {
  if (ks == 1 && gather) return 0;
  if ((ks == 3 || ks == 1) && H == x6t::H && W == x6t::W && Cin == x6t::CIN && (Cout == 256 || Cout == 128)) return 1;
  // the pre-split tiles (conv_x6p_kernel<.., NP = 2>): contiguous 3x3 convs where an x3 instance exists (the 16x20 and
  // 8x10 representation convs)
  return ks == 3 && !gather && H >= 2 && W >= 2 &&
                 x3_halo_launch(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1, H, W, Cin, Cout, 1, nullptr, true) == 0
             ? 1
             : 0;
}

int mzba_conv_x3_ex(const void* in, long long env_stride, const int32_t* slot, long long slot_stride, const void* wx3,
                    const float* wscale, const float* bias, const float* act_bias, const int32_t* act, int A,
                    const void* res, void* out, int B, int H, int W, int Cin, int Cout, int ks, int relu,
                    hipStream_t stream) {
  MZ_CHECK_ARG(in && wx3 && wscale && bias && out && B > 0, -1);
  MZ_CHECK_ARG(!act_bias || (act && A > 0 && !res), -1);
  const bool ga = slot || act_bias || env_stride != (long long)H * W * Cin;
  MZ_CHECK_ARG(mzba_conv_x3_supported(H, W, Cin, Cout, ks, ga ? 1 : 0), -2);
  MZ_CHECK_ARG((long long)B * H * W + 256 < (1LL << 31), -3);
  if (!(H == x6t::H && W == x6t::W)) {
    const int rc = x3_halo_launch(in, wx3, wscale, bias, res, out, B, H, W, Cin, Cout, relu, stream);
    if (rc == 0) MZ_LAUNCH_CHECK();
    return rc;
  }
  X6TArgs t{(const float*)in, env_stride, slot, slot_stride, (const bf16_t*)wx3, bias, act_bias, act, A,
            (const float*)res, (float*)out, B, Cout, relu, (long long)Cout * ks * ks * Cin, wscale};
  if (g_x3_pipe == 2)
    x6t_launch<2, false>(t, ks, ga, stream, 4);  // two 4-wave workgroups per CU
  else
    g_x3_pipe ? x6t_launch<2, true>(t, ks, ga, stream) : x6t_launch<2, false>(t, ks, ga, stream);
  MZ_LAUNCH_CHECK();
  return 0;
}

// out = act(conv3x3(in) + bias (+ res)) in f32 on contiguous NHWC images of B envs, every product as the
// six split-bf16 terms (above); wx = the three bf16 parts of the f32 [Cout][3][3][Cin] weights, each in the
// pack_lat16 packing, back to back (agent.py PackedNets._conv "wx").
int mzba_conv_x6(const void* in, const void* wx, const float* bias, const void* res, void* out, int B, int H, int W,
                 int Cin, int Cout, int relu, hipStream_t stream) {
  return mzba_conv_x6_ex(in, (long long)H * W * Cin, nullptr, 0, wx, bias, nullptr, nullptr, 0, res, out, B, H, W, Cin,
                         Cout, 3, relu, stream);
}

}  // extern "C"

namespace {
// the halo-staged forms (conv_x6p_kernel, else conv_x6_kernel) on contiguous images, Cout % 256 == 0
int x6_halo_launch(const void* in, const void* wx, const float* bias, const void* res, void* out, int B, int H, int W,
                   int Cin, int Cout, int relu, hipStream_t stream) {
  const long long M = (long long)B * H * W;
  MZ_CHECK_ARG(M + 256 < (1LL << 31), -3);  // pixel indices in int (global offsets are size_t)
  X6Args a{(const float*)in, (const bf16_t*)wx, bias, (const float*)res, (float*)out, (int)M, H, W, Cin, Cout, relu};
  a.part = (long long)Cout * 9 * Cin;
  X6Args ap = a;
  // the pre-split form (the Cout 128 instance has no per-read-split twin: taken whatever the A/B variant)
  const X6PGeo geo = (g_x6_variant >= 1 || Cout == 128) ? x6p_geometry(W, Cin, Cout, M, ap) : X6PGeo{};
  const int tmp = geo.tm;
  if (tmp) {
    const int ldsp = ap.ZOFF + 3 * (Cin / geo.nblk) * 2;
    const dim3 gridp((unsigned)((M + tmp - 1) / tmp), (unsigned)(Cout / (128 * geo.ct)));
    auto launchp = [&](auto kern) {
      mz_set_lds_max_once(reinterpret_cast<const void*>(kern), x6::LDS_MAX);
      hipLaunchKernelGGL(kern, gridp, dim3(x6::NT), ldsp, stream, ap);
    };
    if (tmp == 160) {  // the 16x20 instances
      if (Cin == 256)
        launchp(conv_x6p_kernel<256, 160, 2, 2>);
      else if (geo.ct == 2)
        launchp(conv_x6p_kernel<128, 160, 2, 1>);
      else
        launchp(conv_x6p_kernel<128, 160, 1, 1>);
    } else if (Cin == 256) {
      switch (tmp) {
        case 128: launchp(conv_x6p_kernel<256, 128>); break;
        case 112: launchp(conv_x6p_kernel<256, 112>); break;
        case 96: launchp(conv_x6p_kernel<256, 96>); break;
        case 80: launchp(conv_x6p_kernel<256, 80>); break;
        case 64: launchp(conv_x6p_kernel<256, 64>); break;
        default: launchp(conv_x6p_kernel<256, 48>); break;
      }
    } else {
      switch (tmp) {
        case 128: launchp(conv_x6p_kernel<128, 128>); break;
        case 112: launchp(conv_x6p_kernel<128, 112>); break;
        case 96: launchp(conv_x6p_kernel<128, 96>); break;
        case 80: launchp(conv_x6p_kernel<128, 80>); break;
        case 64: launchp(conv_x6p_kernel<128, 64>); break;
        default: launchp(conv_x6p_kernel<128, 48>); break;
      }
    }
    MZ_LAUNCH_CHECK();
    return 0;
  }
  X6Args g0{};
  MZ_CHECK_ARG(Cout % 256 == 0 && H >= 2 && W >= 2 && x6_geometry(W, Cin, g0) > 0, -2);
  const int tm = x6_geometry(W, Cin, a);
  const int lds = a.ZOFF + 16 * Cin * 4;
  const dim3 grid((unsigned)((M + tm - 1) / tm), (unsigned)(Cout / x6::TN));
  auto launch = [&](auto kern) {
    mz_set_lds_max_once(reinterpret_cast<const void*>(kern), x6::LDS_MAX);
    hipLaunchKernelGGL(kern, grid, dim3(x6::NT), lds, stream, a);
  };
  if (Cin == 256)
    tm == 96 ? launch(conv_x6_kernel<256, 96>) : launch(conv_x6_kernel<256, 64>);
  else
    tm == 96 ? launch(conv_x6_kernel<128, 96>) : launch(conv_x6_kernel<128, 64>);
  MZ_LAUNCH_CHECK();
  return 0;
}

// the x3 form on the pre-split tiles, with a batch-independent choice: W >= 16 (the 16x20 representation convs) 160-pixel
// tiles (Cin 256 in two 128-channel blocks; Cin 128 at Cout 256 or 128); otherwise Cin 256, Cout % 256 == 0 on
// x6p_geometry's tile (two fp16 planes per row instead of three bf16: the x6 tile always fits). -2 elsewhere (dry: the
// check only)
int x3_halo_launch(const void* in, const void* wx3, const float* wscale, const float* bias, const void* res, void* out,
                   int B, int H, int W, int Cin, int Cout, int relu, hipStream_t stream, bool dry) {
  const long long M = (long long)B * H * W;
  MZ_CHECK_ARG(M + 256 < (1LL << 31), -3);
  X6Args ap{(const float*)in, (const bf16_t*)wx3, bias, (const float*)res, (float*)out, (int)M, H, W, Cin, Cout, relu};
  ap.part = (long long)Cout * 9 * Cin;
  ap.wscale = wscale;
  X6PGeo geo{};
  if (W >= 16) {
    const bool ok = (Cin == 256 && Cout % 256 == 0) || (Cin == 128 && (Cout % 256 == 0 || Cout == 128));
    geo.tm = 160, geo.nblk = Cin == 256 ? 2 : 1, geo.ct = Cout % 256 == 0 ? 2 : 1;
    if (!ok || (160 + 2 * (W + 1) + 1) * 2 * (Cin / geo.nblk) * 2 > x6::LDS_MAX) return -2;
    ap.HALO = W + 1, ap.NI = 0;
  } else {
    if (Cin != 256 || Cout % 256 != 0) return -2;
    geo = x6p_geometry(W, Cin, Cout, M, ap);
    if (!geo.tm || geo.ct != 2 || geo.nblk != 1) return -2;
  }
  if (dry) return 0;
  const int tm = geo.tm;
  ap.ZOFF = (tm + 2 * (W + 1)) * 2 * (Cin / geo.nblk) * 2;  // HR rows of hi | lo
  const int ldsp = ap.ZOFF + 2 * (Cin / geo.nblk) * 2;
  const dim3 gridp((unsigned)((M + tm - 1) / tm), (unsigned)(Cout / (128 * geo.ct)));
  auto launchp = [&](auto kern) {
    mz_set_lds_max_once(reinterpret_cast<const void*>(kern), x6::LDS_MAX);
    hipLaunchKernelGGL(kern, gridp, dim3(x6::NT), ldsp, stream, ap);
  };
  if (tm == 160) {
    if (Cin == 256)
      launchp(conv_x6p_kernel<256, 160, 2, 2, 2>);
    else if (geo.ct == 2)
      launchp(conv_x6p_kernel<128, 160, 2, 1, 2>);
    else
      launchp(conv_x6p_kernel<128, 160, 1, 1, 2>);
  } else {
    switch (tm) {
      case 128: launchp(conv_x6p_kernel<256, 128, 2, 1, 2>); break;
      case 112: launchp(conv_x6p_kernel<256, 112, 2, 1, 2>); break;
      case 96: launchp(conv_x6p_kernel<256, 96, 2, 1, 2>); break;
      case 80: launchp(conv_x6p_kernel<256, 80, 2, 1, 2>); break;
      case 64: launchp(conv_x6p_kernel<256, 64, 2, 1, 2>); break;
      default: launchp(conv_x6p_kernel<256, 48, 2, 1, 2>); break;
    }
  }
  return 0;
}
}  // namespace

extern "C" {

int mzba_conv_x6_set_variant(int v) {
  if (v < 0 || v > 3) return -1;
  g_x6_variant = v;
  return 0;
}

int mzba_conv_x3_set_pipe(int on) {
  if (on < 0 || on > 2) return -1;
  g_x3_pipe = on;
  return 0;
}

int mzba_conv_x6_set_waves(int nw) {
  if (nw != 0 && nw != 4 && nw != 8) return -1;
  g_x6t_waves = nw;
  return 0;
}

}  // extern "C"
