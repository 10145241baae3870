// Halo-tiled 3x3 convolution for large images (gfx950, bf16 MFMA): config 3's 21x21 latent towers and its
// 42x42 / 84x84 representation convs (networks.py:19-35, 38-241 at the 84x84 / 4-frame geometry).
//
// out[m][n] = act(sum_{tap, c} in[m + dy W + dx][c] W[n][tap][c] + bias[n] (+ res[m][n])), m = (env, y, x)
// flattened over the batch, NHWC bf16, zero padding (taps leaving the image read zeros).
//
// A workgroup (8 waves) owns TM = 256 consecutive output pixels x 256 output
// channels. A 3x3 tap shifts the flattened pixel index by dy W + dx, so every tap of the tile reads rows of ONE
// staged range: the tile's pixels plus a halo of W + 1 rows on each side (HR = 256 + 2 W + 2 pixel rows). That
// range is staged into LDS once, all Cin (128 or 256) channels (supported while HR x 2 Cin B plus the 16-row zero
// block fits the 160 KiB: W <= 23 at Cin 256, W <= 183 at Cin 128; past W = 23 at Cin 256 in two 128-channel
// blocks, up to W = 183; halo_geometry) with LDS-DMA (global_load_lds_dwordx4, no VGPR round trip), and the 9 taps
// x the block's channel steps run from it — the activation operand is fetched from L2 once per tile, not once
// per tap as an im2col GEMM tile fetches it (conv_big_bf16_kernel: 9 x the activation traffic and its LDS
// writes every K step).
//   * LDS row r = pixel m0 - (W + 1) + r, 16-B chunks XOR-swizzled by hkey(r): a B fragment (16
//     consecutive rows = 16 pixels of a tile shifted by any tap, 8 channels per lane) is conflict-free in each
//     of ds_read_b128's four 16-lane groups for every shift (key r & 15, round 3, was 2-way conflicted at odd
//     shifts); LDS-DMA writes lane-linear 1-KiB blocks, so the swizzle is applied on the source addresses.
//     A tap that leaves the image (y + dy or x + dx outside, which the flattened shift wraps into the
//     neighbouring row or env) reads a 16-row zero block instead, at its own row's bank slot.
//   * 8 waves (two per SIMD), each 128 pixels (8 tiles) x 64 output channels (4 column tiles): 32
//     accumulators (128 AGPRs); weights = MFMA A operand from a two-k-step register ring (buffer_load_dwordx4
//     off a wave-uniform resource, the fragment-major packing pack_lat16 of [Cout][tap][Cin]), activations =
//     B operand from LDS (v_mfma_f32_16x16x32_bf16): per 32-channel k step 8 B reads + 4 weight loads feed 32
//     MFMAs, pixel-tile major (each B fragment feeds its 4 MFMAs back to back).
//   * epilogue: + bias (+ residual), ReLU, bf16; a lane holds 4 consecutive channels of one pixel.
//   * Cout 128 (the prediction's 3x3 policy-head conv, networks.py:200-206): TN = 128, 4 pixel quarters x 2
//     channel halves of 64. GA instances (the dynamics' first conv, networks.py:117-122 / agent.py dyn0): the
//     input gathered per env from the latent pool (in + b env_stride + slot[b] slot_stride) and the action
//     planes' contribution added from their folded [HW][A][Cout] table, as conv_igemm ((acc + act_bias) + bias);
//     a staged range then spans at most two envs (HR <= H W), whose offsets are read once per workgroup.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#ifndef HALO_EPI16
#define HALO_EPI16 1  // 16-B epilogue accesses through v_permlane16_swap (0: the round-4 8-B form, an A/B build)
#endif
#ifndef HALO_RING
#define HALO_RING 2  // weight ring depth in k steps (an A/B build may deepen it)
#endif
namespace hl {
constexpr int TM = 256;            // output pixels per workgroup
constexpr int TN = 256;            // output channels per workgroup
constexpr int NT = 512;            // 8 waves, two per SIMD
constexpr int LDS_MAX = 160 * 1024;
}  // namespace hl

struct HaloArgs {
  const bf16_t* in;    // [M][Cin]
  const bf16_t* wh;    // pack_lat16: [Cout / 16][9 Cin / 32][64][8]
  const float* bias;   // [Cout]
  const bf16_t* res;   // optional [M][Cout]
  bf16_t* out;         // [M][Cout]
  int M, H, W, Cin, Cout, relu;
  int HALO, HR, CB;    // halo rows each side, staged rows, channels per staged block
  int NI, ZOFF;        // LDS-DMA 1-KiB blocks per staging, byte offset of the zero block (pipelined: row)
  // GA instances only
  const int32_t* slot;                // optional [B]: env b's input at in + b env_stride + slot[b] slot_stride
  long long env_stride, slot_stride;  // elements
  const float* act_bias;              // optional [H W][A][Cout] f32
  const int32_t* act;                 // [B] (with act_bias)
  int A;
};

// swizzle key of staged row r: ds_read_b128 serves a wave in lane groups {0-3, 12-15, 20-27}, ... (rows
// n = 0-3, 12-15 of k quarter q with rows 4-11 of quarter q ^ 1, MI355X_MICROARCH.md LDS table); with this
// key the 16 chunks (4c + q) ^ key of ANY 16 consecutive rows differ in every group (tools/swizzle_search.py;
// the same key as repblocks.hip's rf::key)
MZ_DEV int hkey(int r) { return ((r << 1) & 6) | (((r >> 2) & 1) * 9); }

// + bias (+ residual), ReLU, bf16: (acc + bias) + res in f32, as conv_big_bf16_kernel; a lane stores 4
// consecutive channels (8 B) of one pixel per (pixel tile, column tile); every residual load of a pixel tile
// is issued before its first use
template <bool RES, bool AB, int MT, int CT>
MZ_DEV void halo_epilogue(const HaloArgs& a, const f32x4 (&acc)[MT][CT], int mb, int nb, int q, int n) {
  const int HW = a.H * a.W;
  // AB: the tile's pixels span at most two envs (TM <= H W): their action indices read once
  int tb0 = 0, tb1 = 0, av0 = 0, av1 = 0;
  if (AB) {
    // a wave wholly past the last pixel (the grid's partial last tile) takes the last env: its clamped pixels
    // (mc = M - 1) then sit in env tb0 and act[] is read in bounds (mb / HW = B read act[B] and indexed with it)
    tb0 = __builtin_amdgcn_readfirstlane(min(mb / HW, a.M / HW - 1));
    tb1 = (tb0 + 1) * HW;
    av0 = a.act[tb0];
    av1 = a.act[min(tb0 + 1, a.M / HW - 1)];
  }
  float4 bb[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) bb[ct] = *reinterpret_cast<const float4*>(a.bias + nb + ct * 16 + 4 * q);
  const float lo = a.relu ? 0.f : -__builtin_inff();  // ReLU as max(v, 0); max(v, -inf) = v
#if HALO_EPI16
  // 16-B form: the k-quarter rows q = 2j and 2j + 1 of a wave hold the two 8-B halves of chunk j (channels 8j..8j + 7
  // of a 16-channel column tile) of the same pixel. For a column-tile pair (ct, ct + 1) one v_permlane16_swap per
  // dword of (acc + bias) hands the odd row's ct half to the even row and the even row's ct + 1 half to the odd
  // row: an even-row lane then owns tile ct's chunk j, an odd-row lane tile ct + 1's, and its residual load, the
  // ReLU / bf16 pack and the store are one 16-B access each (half the epilogue's memory instructions). The f32
  // expression of every element is unchanged, so the outputs are bit-identical to the 8-B form.
  static_assert(CT % 2 == 0, "column-tile pairs");
  const int cj = 8 * (q >> 1), codd = q & 1;
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = mb + mi * 16 + n;
    const int mc = m < a.M ? m : a.M - 1;
    float4 ab[CT];
    if (AB) {
      const bool hi = mc >= tb1;
      const int p = mc - (hi ? tb1 : tb1 - HW), av = hi ? av1 : av0;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        ab[ct] = *reinterpret_cast<const float4*>(a.act_bias + ((size_t)p * a.A + av) * a.Cout + nb + ct * 16 + 4 * q);
    }
    uint4 rv[CT / 2];
    if (RES) {
#pragma unroll
      for (int cp = 0; cp < CT / 2; ++cp)
        rv[cp] = *reinterpret_cast<const uint4*>(a.res + (size_t)mc * a.Cout + nb + (2 * cp + codd) * 16 + cj);
    }
#pragma unroll
    for (int cp = 0; cp < CT / 2; ++cp) {
      float w[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c0 = 2 * cp, c1 = 2 * cp + 1;
        const float v0 = AB ? (acc[mi][c0][i] + (&ab[c0].x)[i]) + (&bb[c0].x)[i] : acc[mi][c0][i] + (&bb[c0].x)[i];
        const float v1 = AB ? (acc[mi][c1][i] + (&ab[c1].x)[i]) + (&bb[c1].x)[i] : acc[mi][c1][i] + (&bb[c1].x)[i];
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v0), __float_as_uint(v1), false, false);
        w[i] = __uint_as_float(r[0]);
        w[4 + i] = __uint_as_float(r[1]);
      }
      if (RES) {
        const uint32_t rw[4] = {rv[cp].x, rv[cp].y, rv[cp].z, rv[cp].w};
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = w[i] + bf16_to_f32((bf16_t)(rw[i >> 1] >> (16 * (i & 1))));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = fmaxf(w[i], lo);
      const uint4 o = make_uint4(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]), pack_bf16x2(w[4], w[5]),
                                 pack_bf16x2(w[6], w[7]));
      if (m < a.M) *reinterpret_cast<uint4*>(a.out + (size_t)m * a.Cout + nb + (2 * cp + codd) * 16 + cj) = o;
    }
  }
#else
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = mb + mi * 16 + n;
    const int mc = m < a.M ? m : a.M - 1;
    uint2 rv[CT];
    float4 ab[CT];
    if (AB) {
      const bool hi = mc >= tb1;
      const int p = mc - (hi ? tb1 : tb1 - HW), av = hi ? av1 : av0;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        ab[ct] = *reinterpret_cast<const float4*>(a.act_bias + ((size_t)p * a.A + av) * a.Cout + nb + ct * 16 + 4 * q);
    }
    if (RES) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) rv[ct] = *reinterpret_cast<const uint2*>(a.res + (size_t)mc * a.Cout + nb + ct * 16 + 4 * q);
    }
    uint2 o[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = AB ? (acc[mi][ct][i] + (&ab[ct].x)[i]) + (&bb[ct].x)[i] : acc[mi][ct][i] + (&bb[ct].x)[i];
      if (RES) {
        v[0] = v[0] + bf16_to_f32((bf16_t)(rv[ct].x & 0xffffu));
        v[1] = v[1] + bf16_to_f32((bf16_t)(rv[ct].x >> 16));
        v[2] = v[2] + bf16_to_f32((bf16_t)(rv[ct].y & 0xffffu));
        v[3] = v[3] + bf16_to_f32((bf16_t)(rv[ct].y >> 16));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], lo);
      o[ct] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
    if (m < a.M) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) *reinterpret_cast<uint2*>(a.out + (size_t)m * a.Cout + nb + ct * 16 + 4 * q) = o[ct];
    }
  }
#endif
}

// WM = 2 pixel halves x 4 quarters of 64 channels. Measured and dropped (profiles/r04/halo_wm/, same box, B = 4096,
// 21x21): WM = 1 (8 slices of 32 channels over all 256 pixels: no weight fragment loaded twice per workgroup,
// half the per-CU L2 weight stream, twice the B reads) 1.76-1.85 ms vs 1.75-1.83; B fragments read 16 MFMAs
// ahead instead of 8: 1.82-1.83 ms. Neither the weight stream nor the LDS read latency bounds this kernel.
// TMW: output pixels per workgroup; OCC: workgroups per CU the register budget allows (2: the 128-pixel instance,
// <= 128 VGPRs at 8 waves, two 128-channel staged blocks of ~44 KiB, so two workgroups share a CU and one's staging
// and epilogue run beside the other's k loop); PFX > 0 sets the fragment read-ahead directly.
template <int CB, int NBLK, int WM = 2, int PFM = 1, int TN = hl::TN, bool GA = false, int NW = 8, int TMW = hl::TM,
          int OCC = 1, int PFX = 0>
__global__ __launch_bounds__(64 * NW, OCC == 1 ? 1 : OCC * NW / 4) void conv_halo_kernel(HaloArgs a) {
  constexpr int RB = CB * 2;        // bytes per staged row
  constexpr int NC = CB / 8;        // 16-B chunks per row
  constexpr int NCS = CB / 32;      // 32-channel k steps per tap and block
  constexpr int WN = NW / WM, CT = TN / 16 / WN, MT = TMW / 16 / WM;  // channel slices, column / pixel tiles per wave
  constexpr int NT = 64 * NW;
  constexpr int PF = PFX > 0 ? PFX : PFM * 8 / CT;  // fragment reads ahead: 8 PFM MFMAs
  static_assert(NCS % 2 == 0, "ring slot = channel step parity");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;  // pixel part (TM / WM), channel slice (16 CT)
  const int q = lane >> 4, n = lane & 15;
  const int m0 = blockIdx.x * TMW, n0 = blockIdx.y * TN;
  const int HW = a.H * a.W;
  // GA: element offset of staged row m = eoff[m >= sb1] + m Cin (the range's two envs, b env_stride + slot[b]
  // slot_stride - b H W Cin)
  long long eoff0 = 0, eoff1 = 0;
  int sb1 = 0;
  if (GA) {
    const int sb0 = __builtin_amdgcn_readfirstlane(max(m0 - a.HALO, 0) / HW), sbn = min(sb0 + 1, a.M / HW - 1);
    sb1 = (sb0 + 1) * HW;
    eoff0 = (long long)sb0 * a.env_stride + (a.slot ? (long long)a.slot[sb0] * a.slot_stride : 0) - (long long)sb0 * HW * a.Cin;
    eoff1 = (long long)sbn * a.env_stride + (a.slot ? (long long)a.slot[sbn] * a.slot_stride : 0) - (long long)sbn * HW * a.Cin;
  }
  const int KS = 9 * a.Cin / 32;            // k steps of the whole conv (pack stride per column tile)
  constexpr int nsteps = NBLK * 9 * NCS;  // NBLK = Cin / CB

  // the zero block: 16 rows (never overwritten by staging)
  for (int i = tid; i < RB; i += NT) *reinterpret_cast<uint4*>(lds + a.ZOFF + i * 16) = make_uint4(0, 0, 0, 0);

  // per pixel tile mi of the wave: the lane's pixel is staged row prow0 + 16 mi at tap (0, 0); byte mi of
  // okw[mi / 4] says which taps stay in the image (bit 0: y > 0, 1: y < H - 1, 2: x > 0, 3: x < W - 1,
  // 4: the pixel exists — rows past M read only the zero block)
  int prow0 = wm * (TMW / WM) + n + a.HALO;
  uint32_t okw[MT / 4] = {};
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m0 + wm * (TMW / WM) + mi * 16 + n;
    if (m < a.M) {
      const int p = m % HW, y = p / a.W, x = p - y * a.W;
      const uint32_t b = 16u | (y > 0 ? 1u : 0u) | (y < a.H - 1 ? 2u : 0u) | (x > 0 ? 4u : 0u) | (x < a.W - 1 ? 8u : 0u);
      okw[mi >> 2] |= b << (8 * (mi & 3));
    }
  }

  // weight ring: k step j (loop order block, tap, channel step) -> pack k step
  auto kstep = [&](int j) {
    j = j < nsteps ? j : nsteps - 1;  // the ring's prefetch past the end re-reads the last step
    const int blk = j / (9 * NCS), r = j - blk * 9 * NCS, t = r / NCS, c = r - t * NCS;
    return t * (a.Cin / 32) + blk * NCS + c;
  };
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(reinterpret_cast<const uint4*>(a.wh) + (size_t)(n0 / 16 + wn * CT) * KS * 64), 0, 0x7fffffff,
      0x00020000);
  auto wload = [&](int ct, int s) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, (ct * KS + s) * 1024, 0));
  };
  bf16x8 bq[HALO_RING][CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int i = 0; i < HALO_RING; ++i) bq[i][ct] = wload(ct, kstep(i));

  f32x4 acc[MT][CT];
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      acc[mi][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  // B fragment of pixel tile mi, channel step c (32 channels: chunk 4c + q of the row) of tap t, its address
  // computed at the read (the tap's shift is wave-uniform; per-tap offset arrays cost 2 MT registers). A lane
  // whose tap leaves the image reads row (r & 15) of a 16-row zero block at ZOFF (16-row aligned): the bank slot
  // its own row would take. One shared zero row put that lane on a slot one of the 15 others held in ~7/8 of
  // such fragments (SQ_LDS_BANK_CONFLICT 0.31 of LDS-active cycles in config 3, profiles/r04/r4f)
  auto frag = [&](int t, int c, int mi) {
    const int dy = t / 3 - 1, dx = t % 3 - 1;
    const uint32_t need = 16u | (dy < 0 ? 1u : 0u) | (dy > 0 ? 2u : 0u) | (dx < 0 ? 4u : 0u) | (dx > 0 ? 8u : 0u);
    const bool ok = ((okw[mi >> 2] >> (8 * (mi & 3))) & need) == need;
    const int r = prow0 + 16 * mi + dy * a.W + dx;
    const int rb = ok ? r * RB : a.ZOFF + (r & 15) * RB;  // the zero block's row with this row's key
    const int key = hkey(r & 15);
    return *reinterpret_cast<const bf16x8*>(lds + rb + (((4 * c + q) ^ key) << 4));
  };
  constexpr int NF = MT * NCS;  // fragments per tap, in (channel step, pixel tile) order

  int j = 0;  // k step
#pragma unroll
  for (int blk = 0; blk < NBLK; ++blk) {
    if (blk > 0) __syncthreads();  // every wave is done with the previous block's rows
    if (NBLK > 1) {  // opaque per block: the fragment addresses CSE'd across the unrolled blocks spilled 322 VGPRs
      asm volatile("" : "+v"(prow0));
#pragma unroll
      for (int i = 0; i < MT / 4; ++i) asm volatile("" : "+v"(okw[i]));
    }
    // stage rows [m0 - HALO, m0 - HALO + HR) x channels [blk CB, (blk + 1) CB): block i of 1 KiB holds
    // chunks 64 i .. 64 i + 63 (row g / NC, physical chunk g % NC = logical chunk ^ hkey(row))
    for (int i = wave; i < a.NI; i += NW) {
      const int g = i * 64 + lane, r = g / NC, s = g - r * NC;
      int m = m0 - a.HALO + r;
      m = m < 0 ? 0 : (m >= a.M ? a.M - 1 : m);  // rows outside [0, M) are only read by masked taps
      const long long eo = GA ? (m >= sb1 ? eoff1 : eoff0) : 0;
      const bf16_t* src = a.in + (eo + (long long)m * a.Cin) + blk * CB + ((s ^ hkey(r)) << 3);
      __builtin_amdgcn_global_load_lds(src, lds + i * 1024, 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bf16x8 fr[2 * PF];  // rolling fragment buffer, PF reads ahead
#pragma unroll
    for (int i = 0; i < PF; ++i) fr[i] = frag(0, 0, i);
    // the taps unrolled: loop-carried accumulators in a rolled loop were renamed and copied between the
    // register files on every iteration
#pragma unroll
    for (int t = 0; t < 9; ++t) {
#pragma unroll
      for (int c = 0; c < NCS; ++c) {
        const int sl = HALO_RING == 2 ? (c & 1) : j % HALO_RING;  // j & 1: the steps per tap (NCS) are even
        const int sn = kstep(j + HALO_RING);
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          const int idx = c * MT + mi, nx = idx + PF;
          if (nx < NF)
            fr[nx % (2 * PF)] = frag(t, nx / MT, nx % MT);
          else if (t < 8)  // the next tap's first fragments (not across a restaging)
            fr[nx % (2 * PF)] = frag(t + 1, (nx - NF) / MT, (nx - NF) % MT);
          const bf16x8 f = fr[idx % (2 * PF)];
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) acc[mi][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[sl][ct], f, acc[mi][ct], 0, 0, 0);
        }
        // this step's ring slots are free once its MFMAs have issued: the step after next
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) bq[sl][ct] = wload(ct, sn);
        // per pixel tile: its fragment read PF tiles ahead, then its CT MFMAs; the ring loads after the step's
        // MFMAs (their slots are free then; issued earlier they would need fresh registers)
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, CT, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, CT, 0);
        __builtin_amdgcn_sched_barrier(0);
        ++j;
      }
    }
  }

  // epilogue: acc[mi][ct] = D[channel n0 + 16 CT wn + 16 ct + 4q + i][pixel m0 + TM / WM wm + 16 mi + n]
  if (GA && a.act_bias)
    halo_epilogue<false, GA>(a, acc, m0 + wm * (TMW / WM), n0 + wn * 16 * CT, q, n);
  else if (a.res)
    halo_epilogue<true, false>(a, acc, m0 + wm * (TMW / WM), n0 + wn * 16 * CT, q, n);
  else
    halo_epilogue<false, false>(a, acc, m0 + wm * (TMW / WM), n0 + wn * 16 * CT, q, n);
}

// staging geometry for a (W, Cin) pair: the whole Cin staged at once where it fits (one block), else Cin 256 in two
// 128-channel blocks (the blocks unrolled: a rolled loop would carry the accumulators across its back edge, which
// the compiler renames and copies); 0 if the halo does not fit the LDS
int halo_geometry(int W, int Cin, HaloArgs& g, int tm = hl::TM, int cb_max = 256) {
  for (int cb = Cin < cb_max ? Cin : cb_max; cb >= 128; cb /= 2) {
    const int halo = W + 1, hr = tm + 2 * halo, rb = cb * 2;
    const int ni = (hr * rb + 1023) / 1024;
    const int zoff = (ni * 1024 + 16 * rb - 1) / (16 * rb) * (16 * rb);  // the 16-row zero block, 16-row aligned
    if ((Cin != 128 && Cin != 256) || zoff + 16 * rb > hl::LDS_MAX) continue;
    g.HALO = halo, g.HR = hr, g.CB = cb, g.NI = ni, g.ZOFF = zoff;
    return zoff + 16 * rb;
  }
  return 0;
}

}  // namespace

static int g_halo_waves = 0;
static int g_halo_form = 0;

extern "C" {

// waves per workgroup of the Cin 256 one-block instances (config 3's 21x21 convs): 0 default (8: two per SIMD, each
// 128 pixels x 64 channels), 4 (one per SIMD, 128 pixels x 128 channels: half the LDS fragment reads per MFMA), 8
int mzba_conv_halo_set_waves(int nw) {
  if (nw != 0 && nw != 4 && nw != 8) return -1;
  g_halo_waves = nw;
  return 0;
}

// pixels per workgroup of the Cin 256 / Cout 256 instances. The 256-pixel form stages all 256 input channels at once
// (one workgroup per CU) where its halo fits the LDS (W <= 23), else two 128-channel blocks; the 128-pixel form (8
// waves of 128 pixels x 32 channels, two staged 128-channel blocks of <= 80 KiB, <= 128 VGPRs: two workgroups per CU,
// one's staging / epilogue beside the other's k loop) takes each output's taps in the two-block order.
// 0 (default): the 128-pixel form where the 256-pixel form would stage two blocks anyway (W > 23: config 3's 42x42
// and 84x84 256-channel convs) — the same k order, so the same bits; 1: the 128-pixel form wherever it fits (the
// 21x21 convs too: block order, bf16-rounding-level differences; measured slower there, profiles/r06/halo_form/);
// 2: never (the round-5 kernels, A/B reference).
int mzba_conv_halo_set_form(int f) {
  if (f < 0 || f > 2) return -1;
  g_halo_form = f;
  return 0;
}

int mzba_conv_halo_supported(int H, int W, int Cin, int Cout, int ks) {
  HaloArgs g{};
  if (ks != 3 || H < 2 || W < 2 || (Cin != 128 && Cin != 256) || halo_geometry(W, Cin, g) == 0) return 0;
  return Cout % 256 == 0 || (Cout == 128 && g.CB == Cin) ? 1 : 0;  // Cout 128: one staged block
}

// gather = 1: a slot-gathered / strided input and / or an action-bias table (the GA instance: Cin 256, Cout % 256
// == 0, the staged range within two envs)
int mzba_conv_halo_ex_supported(int H, int W, int Cin, int Cout, int ks, int gather) {
  if (!mzba_conv_halo_supported(H, W, Cin, Cout, ks)) return 0;
  if (!gather) return 1;
  HaloArgs g{};
  halo_geometry(W, Cin, g);
  return Cin == 256 && g.CB == 256 && Cout % 256 == 0 && g.HR <= H * W ? 1 : 0;
}

// out = act(conv3x3(in, W) (+ act_bias[p][act[b]]) + bias (+ res)); env b's input image at in + b env_stride +
// slot[b] slot_stride (slot optional; env_stride = H W Cin with neither slot nor act_bias: contiguous); wh = the
// pack_lat16 packing of the BN-folded [Cout][3][3][Cin] weights (agent.py PackedNets._conv "wh").
int mzba_conv_halo_ex(const void* in, long long env_stride, const int32_t* slot, long long slot_stride, const void* wh,
                      const float* bias, const float* act_bias, const int32_t* act, int A, const void* res, void* out,
                      int B, int H, int W, int Cin, int Cout, int relu, hipStream_t stream) {
  MZ_CHECK_ARG(in && wh && bias && out && B > 0, -1);
  MZ_CHECK_ARG(!act_bias || (act && A > 0 && !res), -1);
  const bool ga = slot || act_bias || env_stride != (long long)H * W * Cin;
  MZ_CHECK_ARG(mzba_conv_halo_ex_supported(H, W, Cin, Cout, 3, ga ? 1 : 0), -2);
  const long long M = (long long)B * H * W;
  MZ_CHECK_ARG(M + 2 * hl::TM < (1LL << 31), -3);  // pixel indices in int (global offsets are size_t)
  HaloArgs a{(const bf16_t*)in, (const bf16_t*)wh, bias, (const bf16_t*)res, (bf16_t*)out, (int)M, H, W, Cin, Cout, relu};
  a.slot = slot, a.env_stride = env_stride, a.slot_stride = slot_stride, a.act_bias = act_bias, a.act = act, a.A = A;
  const int tn = Cout % 256 == 0 ? 256 : 128;
  typedef void (*Kern)(HaloArgs);
  HaloArgs g0{};
  const bool two_blocks = halo_geometry(W, Cin, g0) > 0 && g0.CB < Cin;  // the 256-pixel form's staging
  if (Cin == 256 && tn == 256 && (g_halo_form == 1 || (g_halo_form == 0 && two_blocks && !ga))) {  // 128-pixel form
    HaloArgs g{};
    const int lds1 = halo_geometry(W, Cin, g, 128, 128);
    if (lds1 > 0 && lds1 <= 80 * 1024 && g.CB == 128 && (!ga || g.HR <= H * W)) {
      a.HALO = g.HALO, a.HR = g.HR, a.CB = g.CB, a.NI = g.NI, a.ZOFF = g.ZOFF;
      static const Kern k1[2] = {conv_halo_kernel<128, 2, 1, 1, 256, false, 8, 128, 2, 2>,
                                 conv_halo_kernel<128, 2, 1, 1, 256, true, 8, 128, 2, 2>};
      static const bool attrs1 = [] {
        for (Kern k : k1)
          (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
        return true;
      }();
      (void)attrs1;
      const dim3 grid1((unsigned)((M + 127) / 128), (unsigned)(Cout / 256));
      hipLaunchKernelGGL(k1[ga ? 1 : 0], grid1, dim3(hl::NT), lds1, stream, a);
      MZ_LAUNCH_CHECK();
      return 0;
    }
  }
  const int lds = halo_geometry(W, Cin, a);
  const dim3 grid((unsigned)((M + hl::TM - 1) / hl::TM), (unsigned)(Cout / tn));
  static const Kern kerns[8] = {conv_halo_kernel<256, 1, 2, 1, 256, true>, conv_halo_kernel<256, 1, 4, 1, 128>,
                                conv_halo_kernel<256, 1>, conv_halo_kernel<128, 1>, conv_halo_kernel<128, 2>,
                                conv_halo_kernel<128, 1, 4, 1, 128>, conv_halo_kernel<256, 1, 2, 1, 256, true, 4>,
                                conv_halo_kernel<256, 1, 2, 1, 256, false, 4>};
  static const bool attrs = [] {  // every instance: the 160 KiB of dynamic LDS
    for (Kern k : kerns)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, hl::LDS_MAX);
    return true;
  }();
  (void)attrs;
  const bool w4 = g_halo_waves == 4;  // the Cin 256 one-block instances: 4 waves of 128 pixels x 128 channels
  const Kern kern = ga ? kerns[w4 ? 6 : 0]
                       : tn == 128 ? (Cin == 256 ? kerns[1] : kerns[5])
                                   : (a.CB == 256 ? kerns[w4 ? 7 : 2] : (Cin == 128 ? kerns[3] : kerns[4]));
  const int nt = w4 && tn == 256 && a.CB == 256 ? 256 : hl::NT;
  hipLaunchKernelGGL(kern, grid, dim3(nt), lds, stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

// the contiguous form (no gather, no action bias)
int mzba_conv_halo(const void* in, const void* wh, const float* bias, const void* res, void* out, int B, int H, int W,
                   int Cin, int Cout, int relu, hipStream_t stream) {
  return mzba_conv_halo_ex(in, (long long)H * W * Cin, nullptr, 0, wh, bias, nullptr, nullptr, 0, res, out, B, H, W, Cin,
                           Cout, relu, stream);
}

}  // extern "C"
