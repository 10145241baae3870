// Representation-net convs at the full 16x20 resolution (bf16, gfx950 MFMA): "band" kernel.
//
// RepresentationNetwork runs 3x3 convs 128->128, 128->256 and 256->256 at 16x20 (networks.py:38-99;
// ConvBlock / ResidualBlock :7-35), M = B*320 rows. A workgroup owns one env and 10 output columns
// x0..x0+9 (160 rows) x all Cout channels:
//   * the input band (12 columns x0-1..x0+10, zero outside the image, x all 16 rows x Cin) is staged
//     once into LDS; LDS row = 16 j + y for source column j. A 16-row MFMA tile is one image COLUMN,
//     so a tap (dy, dx) maps output column t to source column t + 1 + dx whole and shifts rows by dy
//     inside it; rows leaving 0..15 read a 16-row zero block;
//   * weights are the MFMA A operand (pack: agent.pack_tower_conv, taps (dx, dy)), activations the
//     B operand: B column j of every tile carries image row SIG[j], and LDS row y has its 16-B
//     chunks XOR-swizzled by KEY[y]. (SIG, KEY) is a pair for which every ds_read_b128 lane group
//     hits 16 distinct bank slots for all three row shifts (found by search; 16x20's 1-row shifts
//     defeat the plain row-XOR swizzle);
//   * 4 waves (one per SIMD), each all 10 column tiles x Cout/64 channel tiles: every weight fragment
//     fetched from L2 feeds 10 MFMAs;
//   * epilogue through LDS: + bias (+ residual staged coalesced), optional ReLU, bf16, then coalesced
//     16-B stores.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BH = 16, BW = 20;      // image
constexpr int BNT = 256;             // 4 waves
constexpr unsigned long long SIG = 0x93f5a4260ce8b7d1ull;  // nibble j: image row of B column j
constexpr unsigned long long KEY = 0x35a0e1879df426bcull;  // nibble y: swizzle key of image row y

MZ_DEV int nib(unsigned long long t, int i) { return (int)((t >> (4 * i)) & 15); }

// 16-B weight fragment of k step `step` of column tile `ct` (TNS k steps per tile), this lane
template <int TNS>
MZ_DEV uint4 wld(__amdgpu_buffer_rsrc_t rs, int ct, int step, int lane) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (ct * TNS + step) * 1024, 0));
}

struct BandArgs {
  const bf16_t* in;   // [B][320][Cin]
  const bf16_t* wf;   // tower packing [Cout/16][9*Cin/32][64][8] (+ pad)
  const float* bias;  // [Cout]
  const bf16_t* res;  // optional [B][320][Cout]
  bf16_t* out;        // [B][320][Cout]
  int B, relu;
};

#ifndef BAND_ONEPASS
#define BAND_ONEPASS 1  // 0: the three per-shift k loops (band_dx) everywhere, for A/B builds
#endif
#ifndef BAND_ONEPASS128
#define BAND_ONEPASS128 1  // the Cout 128 convs on the one pass too (3-entry ring at 5 columns); 0: A/B build
#endif

#ifdef BAND_STAMPS
// diagnostic build only (make band-stamps -> libmzba_bstamp.so, tools/stamp_band.py): s_memtime at the
// phase boundaries, per workgroup and wave: 0 entry, 1 band staged, 2 k loop done, 3 residual staged,
// 4 epilogue in LDS, 5 exit; 6 / 7 s_memrealtime at entry / exit (100 MHz)
constexpr int BST_N = 8, BST_WG = 8192;
__device__ unsigned long long mz_band_stamps[BST_WG * 4][BST_N];
MZ_DEV void bstamp(int k, bool real = false) {
  if ((threadIdx.x & 63) == 0 && blockIdx.x < BST_WG)
    mz_band_stamps[blockIdx.x * 4 + (threadIdx.x >> 6)][k] =
        real ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
}
#define BSTAMP(k) bstamp(k)
#define BSTAMP_REAL(k) bstamp(k, true)
#else
#define BSTAMP(k) ((void)0)
#define BSTAMP_REAL(k) ((void)0)
#endif

template <int CIN, int COUT, int XT>
struct BandGeo {
  // weight ring depth (k steps; 2 at two workgroups per CU). Ring slot = step % TDB is taken as
  // c % TDB inside a tap, so TDB must divide the NC = Cin / 32 steps of a tap
  static constexpr int TDB = (XT == 10 ? 4 : 2) < CIN / 32 ? (XT == 10 ? 4 : 2) : CIN / 32;
  static_assert((CIN / 32) % TDB == 0, "ring slot restarts at every tap");
  static constexpr int NSRC = XT + 2;              // staged source columns (with the halo)
  // one-pass weight ring (band_all): 3 entries (dx = -1, 0, +1) per k step; two steps in flight, one
  // where two workgroups per CU leave 256 registers per lane for 4 column tiles (6 entries spilled 52)
  static constexpr int RDB = (XT == 5 && (COUT == 256 || BAND_ONEPASS128)) ? 3 : 6;
  // LDS bytes per source row: at Cin 64 the row is padded to 128 channels, so a chunk index XORed
  // with the 4-bit row key stays inside the row (staging and reads use the same mapping; the pad
  // chunks are never read)
  static constexpr int RB = (CIN < 128 ? 128 : CIN) * 2;
  static constexpr int NCH = CIN / 8;              // 16-B chunks per source row (staged)
  static constexpr int NC = CIN / 32;              // k steps per tap
  static constexpr int TNS = 9 * NC;               // k steps per channel tile
  static constexpr int CTW = COUT / 64;            // 16-channel tiles per wave
  static constexpr int OB = COUT * 2;              // LDS bytes per output row
  static constexpr int LZ = NSRC * 16 * RB;        // zero block offset
  static constexpr int IN_BYTES = LZ + 16 * RB;
  static constexpr int OUT_BYTES = XT * 16 * OB;
  static constexpr int BYTES = IN_BYTES > OUT_BYTES ? IN_BYTES : OUT_BYTES;
};

// the 3 dy x NC k steps of column shift DX
template <int CIN, int COUT, int XT, int DX>
__device__ __forceinline__ void band_dx(const uint8_t* __restrict__ lds, __amdgpu_buffer_rsrc_t wrs,
                                        uint4 (&bq)[COUT / 64][BandGeo<CIN, COUT, XT>::TDB], f32x4 (&acc)[XT][COUT / 64],
                                        int lane) {
  using G = BandGeo<CIN, COUT, XT>;
  constexpr int CTW = G::CTW, NC = G::NC, TDB = G::TDB;
  constexpr int SB = (DX + 1) * 3 * NC;
  const int q = lane >> 4, ys = nib(SIG, lane & 15);
  auto rows = [&](int dy, int& base, int& tst, int& sw) {
    const int yy = ys + dy;
    const bool ok = (unsigned)yy < (unsigned)BH;
    base = ok ? ((1 + DX) * 16 + yy) * G::RB : G::LZ + (yy & 15) * G::RB;
    tst = ok ? 16 * G::RB : 0;
    sw = nib(KEY, yy & 15) << 4;
  };
  int base, tst, sw;
  rows(-1, base, tst, sw);
  bf16x8 afc[XT], afn[XT];
#pragma unroll
  for (int t = 0; t < XT; ++t) afc[t] = *reinterpret_cast<const bf16x8*>(lds + base + t * tst + ((q << 4) ^ sw));
#pragma unroll 1
  for (int dyi = 0; dyi < 3; ++dyi) {
    int nbase, ntst, nsw;
    rows(dyi < 2 ? dyi : 1, nbase, ntst, nsw);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int s = SB + dyi * NC + c;
      bf16x8 w[CTW];
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct) {
        w[ct] = __builtin_bit_cast(bf16x8, bq[ct][c % TDB]);
        bq[ct][c % TDB] = wld<G::TNS>(wrs, ct, s + TDB, lane);
      }
#pragma unroll
      for (int t = 0; t < XT; ++t) {
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct)
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[ct], afc[t], acc[t][ct], 0, 0, 0);
        if (c + 1 < NC)
          afn[t] = *reinterpret_cast<const bf16x8*>(lds + base + t * tst + (((4 * (c + 1) + q) << 4) ^ sw));
        else
          afn[t] = *reinterpret_cast<const bf16x8*>(lds + nbase + t * ntst + ((q << 4) ^ nsw));
      }
      // every A read of the next k step in the first XT MFMA slots: the compiler orders a step's
      // independent MFMAs freely, so the next step may open with any tile (tower.hip tower8_dx)
#pragma unroll
      for (int t = 0; t < XT; ++t) {
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, XT * CTW - XT - CTW, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < XT; ++t) afc[t] = afn[t];
    }
    base = nbase; tst = ntst; sw = nsw;
  }
}


// the one pass runs every conv (B = 4096 isolated: 256->256 1202 -> 1131 us, 128->256 675 -> 639 us;
// 128->128 with the 3-entry ring 368 -> 355 us). The Cout 128 convs kept the three loops in round 2
// because their one pass moved the bf16 learner's gradients past a noise bound between two bf16
// realisations; that bound was a lucky seed (tools/learner_bn_calib.py: 0.86 - 0.9998 over 6 seeds on
// either build) and the learner test now checks each realisation against the f32 path instead
template <int COUT> constexpr bool band_one = BAND_ONEPASS && (COUT == 256 || BAND_ONEPASS128);

// pack step of one-pass ring entry e = 3 (dyi * NC + c) + d (d = dx + 1)
template <int NC>
MZ_DEV int band_step(int e) { return (e % 3) * 3 * NC + e / 3; }

// One k-loop pass over all three column shifts (tower.hip tower8_dall): per (dy, channel step) the
// XT + 2 source columns are read from LDS once; output column t takes dx = -1 from source t, dx = 0
// from t + 1, dx = +1 from t + 2. Column-tile major: a column tile's 3 x XT MFMAs, then its three
// ring slots reloaded RDB / 3 steps ahead (free registers once the MFMAs have issued: no copies)
// (the residual-block kernel runs it on a wider staged band: source columns from byte offset CB of the
// LDS image, the zero block after LZC staged columns)
template <int CIN, int COUT, int XT, int LZC = XT + 2, int CB = 0, int ACC = XT, int RDB = BandGeo<CIN, COUT, XT>::RDB>
__device__ __forceinline__ void band_all(const uint8_t* __restrict__ lds, __amdgpu_buffer_rsrc_t wrs,
                                         uint4 (&bq)[COUT / 64][RDB], f32x4 (&acc)[ACC][COUT / 64], int lane) {
  static_assert(ACC >= XT, "accumulator rows");
  using G = BandGeo<CIN, COUT, XT>;
  constexpr int CTW = G::CTW, NC = G::NC, NS = XT + 2;
  constexpr int LZ = LZC * 16 * G::RB;
  static_assert((3 * NC) % RDB == 0 && 3 * XT >= NS, "ring slot restarts at every dy; schedule groups");
  const int q = lane >> 4, ys = nib(SIG, lane & 15);
  auto rows = [&](int dy, int& base, int& tst, int& sw) {
    const int yy = ys + dy;
    const bool ok = (unsigned)yy < (unsigned)BH;
    base = ok ? CB + yy * G::RB : LZ + (yy & 15) * G::RB;
    tst = ok ? 16 * G::RB : 0;
    sw = nib(KEY, yy & 15) << 4;
  };
  int base, tst, sw;
  rows(-1, base, tst, sw);
  bf16x8 afc[NS], afn[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) afc[j] = *reinterpret_cast<const bf16x8*>(lds + base + j * tst + ((q << 4) ^ sw));
#pragma unroll 1
  for (int dyi = 0; dyi < 3; ++dyi) {
    int nbase, ntst, nsw;
    rows(dyi < 2 ? dyi : 1, nbase, ntst, nsw);
    const bool last = dyi == 2;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct) {
        bf16x8 w[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) w[d] = __builtin_bit_cast(bf16x8, bq[ct][(3 * c + d) % RDB]);
#pragma unroll
        for (int t = 0; t < XT; ++t) acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], afc[t + 1], acc[t][ct], 0, 0, 0);
        if (ct == 0) {
#pragma unroll
          for (int j = 0; j < NS; ++j) {
            if (c + 1 < NC)
              afn[j] = *reinterpret_cast<const bf16x8*>(lds + base + j * tst + (((4 * (c + 1) + q) << 4) ^ sw));
            else
              afn[j] = *reinterpret_cast<const bf16x8*>(lds + nbase + j * ntst + ((q << 4) ^ nsw));
          }
        }
#pragma unroll
        for (int t = 0; t < XT; ++t) acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], afc[t], acc[t][ct], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < XT; ++t) acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], afc[t + 2], acc[t][ct], 0, 0, 0);
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          // RDB / 3 steps ahead (pack step 3 NC d + dyi NC + c + RDB / 3); past the conv's end (dy = +1,
          // last channel steps) the current step is re-read instead (in range, never used)
          const int nxt = (ct * G::TNS + d * 3 * NC + dyi * NC + c + RDB / 3) * 1024;
          const int cur = (ct * G::TNS + d * 3 * NC + dyi * NC + c) * 1024;
          const int so = (c + RDB / 3 >= NC && last) ? cur : nxt;
          bq[ct][(3 * c + d) % RDB] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, so, 0));
        }
        if (ct == 0) {
#pragma unroll
          for (int j = 0; j < NS; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 3 * XT - NS, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 3 * XT, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NS; ++j) afc[j] = afn[j];
    }
    base = nbase; tst = ntst; sw = nsw;
  }
}

// XT output columns per workgroup (10: one workgroup per CU at Cin 256; 5: two per CU, so one
// workgroup's band staging / epilogue runs beside the other's MFMAs)
template <int CIN, int COUT, int XT>
__global__ __launch_bounds__(BNT, XT == 10 ? 1 : 2) void band_conv_kernel(BandArgs a) {
  using G = BandGeo<CIN, COUT, XT>;
  constexpr int NSRC = G::NSRC, NB = BW / XT;
  constexpr int CTW = G::CTW;
  __shared__ __attribute__((aligned(16))) uint8_t lds[G::BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / NB, x0 = (blockIdx.x % NB) * XT;
  BSTAMP_REAL(6);
  BSTAMP(0);
  // stage the band: NSRC*16 rows x NCH chunks, then the zero block. Every load of the band is in
  // flight at once (one memory round trip; batches of 4 per thread behind a `#pragma unroll 1` waited
  // once per batch)
  {
    constexpr int N = NSRC * 16 * G::NCH;
    constexpr int UB = (N + BNT - 1) / BNT;
    constexpr bool EXACT = N % (UB * BNT) == 0;  // else the last batch is partial (guarded)
    const bf16_t* src = a.in + (size_t)b * BH * BW * CIN;
    {
      const int i0 = 0;
      uint4 v[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int i = i0 + u * BNT + tid;
        const int row = i / G::NCH, ch = i % G::NCH;
        const int x = x0 - 1 + (row >> 4), y = row & 15;
        const bool ok = (unsigned)x < (unsigned)BW && (EXACT || i < N);
        v[u] = *reinterpret_cast<const uint4*>(src + ((size_t)(y * BW + (ok ? x : 0)) * CIN + (ok ? ch * 8 : 0)));
        if (!ok) v[u] = make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int i = i0 + u * BNT + tid;
        const int row = i / G::NCH, ch = i % G::NCH;
        if (EXACT || i < N) *reinterpret_cast<uint4*>(lds + row * G::RB + ((ch ^ nib(KEY, row & 15)) << 4)) = v[u];
      }
    }
    for (int i = tid; i < G::RB; i += BNT) *reinterpret_cast<uint4*>(lds + G::LZ + i * 16) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  BSTAMP(1);
  // this wave's column tiles of the weight pack through a wave-uniform buffer resource (one VGPR for
  // the lane offset; the (tile, step) offset in an SGPR)
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(reinterpret_cast<const uint4*>(a.wf) + (size_t)__builtin_amdgcn_readfirstlane(wave * CTW) * G::TNS * 64),
      0, 0x7fffffff, 0x00020000);
  constexpr int TDB = band_one<COUT> ? G::RDB : G::TDB;
  uint4 bq[CTW][TDB];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
    for (int i = 0; i < TDB; ++i) bq[ct][i] = wld<G::TNS>(wrs, ct, band_one<COUT> ? band_step<G::NC>(i) : i, lane);
  f32x4 acc[XT][CTW];
#pragma unroll
  for (int t = 0; t < XT; ++t)
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) acc[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (band_one<COUT>) {
    band_all<CIN, COUT, XT>(lds, wrs, bq, acc, lane);
  } else {
    band_dx<CIN, COUT, XT, -1>(lds, wrs, bq, acc, lane);
    band_dx<CIN, COUT, XT, 0>(lds, wrs, bq, acc, lane);
    band_dx<CIN, COUT, XT, 1>(lds, wrs, bq, acc, lane);
  }
  BSTAMP(2);
  __syncthreads();  // the band is no longer read
  // output tile in LDS: row 16 t + y, 16-B chunks swizzled by KEY[y]
  constexpr int ONCH = COUT / 8;
  bf16_t* gout = a.out + (size_t)b * BH * BW * COUT;
  if (a.res) {  // stage the residual tile (coalesced): every load in flight, then the LDS writes
    const bf16_t* gres = a.res + (size_t)b * BH * BW * COUT;
    constexpr int NR = XT * 16 * ONCH, UR = (NR + BNT - 1) / BNT;
    uint4 rv[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const int i = min(u * BNT + tid, NR - 1);
      const int row = i / ONCH, ch = i % ONCH, t = row >> 4, y = row & 15;
      rv[u] = *reinterpret_cast<const uint4*>(gres + (size_t)(y * BW + x0 + t) * COUT + ch * 8);
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const int i = u * BNT + tid;
      const int row = i / ONCH, ch = i % ONCH, y = row & 15;
      if (NR % BNT == 0 || i < NR) *reinterpret_cast<uint4*>(lds + row * G::OB + ((ch ^ nib(KEY, y)) << 4)) = rv[u];
    }
    __syncthreads();
  }
  BSTAMP(3);
  {
    const int q = lane >> 4, ys = nib(SIG, lane & 15), ky = nib(KEY, ys);
    float4 bias4[CTW];  // every bias load in flight before the first use
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) bias4[ct] = *reinterpret_cast<const float4*>(a.bias + (wave * CTW + ct) * 16 + 4 * q);
    // every residual element of this lane read from LDS before any result is written back: a read
    // after the previous element's write (same array) was one serialised LDS round trip per element
    // (stamps: 13.4 k cycles of epilogue at 256 -> 256)
    uint2 rr[CTW][XT];
    if (a.res) {
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct) {
        const int n = (wave * CTW + ct) * 16 + 4 * q;
#pragma unroll
        for (int t = 0; t < XT; ++t)
          rr[ct][t] = *reinterpret_cast<const uint2*>(lds + (t * 16 + ys) * G::OB + (((n >> 3) ^ ky) << 4) + ((n & 7) << 1));
      }
    }
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) {
      const int n = (wave * CTW + ct) * 16 + 4 * q;  // D[channel n + i][column j = lane & 15]
      const float4 b4 = bias4[ct];
#pragma unroll
      for (int t = 0; t < XT; ++t) {
        uint2* p = reinterpret_cast<uint2*>(lds + (t * 16 + ys) * G::OB + (((n >> 3) ^ ky) << 4) + ((n & 7) << 1));
        float v0 = acc[t][ct][0] + b4.x, v1 = acc[t][ct][1] + b4.y, v2 = acc[t][ct][2] + b4.z, v3 = acc[t][ct][3] + b4.w;
        if (a.res) {
          const uint2 r = rr[ct][t];
          v0 += __uint_as_float(r.x << 16); v1 += __uint_as_float(r.x & 0xffff0000u);
          v2 += __uint_as_float(r.y << 16); v3 += __uint_as_float(r.y & 0xffff0000u);
        }
        if (a.relu) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
        uint2 o;
        o.x = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
        o.y = (uint32_t)f32_to_bf16(v2) | ((uint32_t)f32_to_bf16(v3) << 16);
        *p = o;
      }
    }
  }
  __syncthreads();
  BSTAMP(4);
  for (int i = tid; i < XT * 16 * ONCH; i += BNT) {
    const int row = i / ONCH, ch = i % ONCH, t = row >> 4, y = row & 15;
    *reinterpret_cast<uint4*>(gout + (size_t)(y * BW + x0 + t) * COUT + ch * 8) =
        *reinterpret_cast<const uint4*>(lds + row * G::OB + ((ch ^ nib(KEY, y)) << 4));
  }
  BSTAMP(5);
  BSTAMP_REAL(7);
}

// ResidualBlock(C) at 16x20 (networks.py:19-35; RepresentationNetwork's blocks, :46-92) in ONE launch:
// out = relu(conv2(relu(conv1(x) + b1)) + b2 + x), BN folded. A workgroup owns one env and the 10 output
// columns x0..x0+9 (x0 = 0 or 10): it stages the 14 source columns x0-2..x0+11 once; conv1 computes the
// 12 columns x0-1..x0+10 (the band and the halo conv2 needs; a column outside the image is written as
// zeros, conv2's padding) and writes them back in place as bf16 — what the two-launch sequence stores —
// then conv2 computes the band from them, + bias + the residual (re-read from global), ReLU. The same
// k loop as band_conv_kernel, so the outputs equal two band launches bit for bit; every weight fragment
// feeds 12 (conv1) / 10 (conv2) MFMAs instead of 5, at 10 % recomputed halo columns.
#ifndef BAND_RES_RDB
#define BAND_RES_RDB 3
#endif

struct BandResArgs {
  const bf16_t* in;   // [B][320][C]
  const bf16_t* w1;   // tower packing (+ pad)
  const float* b1;
  const bf16_t* w2;
  const float* b2;
  bf16_t* out;        // [B][320][C]; must not alias in (neighbouring bands read its halo columns)
  int B;
};

template <int C>
__global__ __launch_bounds__(BNT, 1) void band_res_kernel(BandResArgs a) {
  using G1 = BandGeo<C, C, 12>;  // conv1: 12 output tiles over the 14 staged columns
  using G2 = BandGeo<C, C, 10>;  // conv2: 10 output tiles over staged columns 1..12
  // weight ring: 3 entries (one k step) per column tile; the 12 accumulator tiles take 192 of the 256
  // AGPRs at C = 256, the A fragments of two k steps 112 VGPRs
  constexpr int NSRC = 14, CTW = G1::CTW, RB = G1::RB, NC = G1::NC, TNS = G1::TNS, RDB = BAND_RES_RDB;
  static_assert(G2::RB == RB && RB == 2 * C, "one row layout for both convs");
  constexpr int LZ = NSRC * 16 * RB;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LZ + 16 * RB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x >> 1, x0 = (blockIdx.x & 1) * 10;
  BSTAMP_REAL(6);
  BSTAMP(0);
  const bf16_t* src = a.in + (size_t)b * BH * BW * C;
  {  // stage source columns x0-2 .. x0+11 (zero outside the image), every load in flight at once
    constexpr int NCH = C / 8, N = NSRC * 16 * NCH, UB = N / BNT;
    static_assert(N % BNT == 0, "whole batches");
    uint4 v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = u * BNT + tid;
      const int row = i / NCH, ch = i % NCH;
      const int x = x0 - 2 + (row >> 4), y = row & 15;
      const bool ok = (unsigned)x < (unsigned)BW;
      v[u] = *reinterpret_cast<const uint4*>(src + ((size_t)(y * BW + (ok ? x : 0)) * C + ch * 8));
      if (!ok) v[u] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = u * BNT + tid;
      const int row = i / NCH, ch = i % NCH;
      *reinterpret_cast<uint4*>(lds + row * RB + ((ch ^ nib(KEY, row & 15)) << 4)) = v[u];
    }
    for (int i = tid; i < RB; i += BNT) *reinterpret_cast<uint4*>(lds + LZ + i * 16) = make_uint4(0, 0, 0, 0);
  }
  const int wt = __builtin_amdgcn_readfirstlane(wave * CTW);
  const __amdgpu_buffer_rsrc_t wrs1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(reinterpret_cast<const uint4*>(a.w1) + (size_t)wt * TNS * 64), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(reinterpret_cast<const uint4*>(a.w2) + (size_t)wt * TNS * 64), 0, 0x7fffffff, 0x00020000);
  uint4 bq[CTW][RDB];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
    for (int i = 0; i < RDB; ++i) bq[ct][i] = wld<TNS>(wrs1, ct, band_step<NC>(i), lane);
  f32x4 acc[12][CTW];
#pragma unroll
  for (int t = 0; t < 12; ++t)
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) acc[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  BSTAMP(1);
#pragma unroll
  for (int t = 0; t < 12; ++t)  // accumulators in the AGPR half (tower.hip: no per-step copies)
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) asm volatile("" : "+a"(acc[t][ct]));
  band_all<C, C, 12, NSRC, 0, 12, RDB>(lds, wrs1, bq, acc, lane);
  const int q = lane >> 4, ys = nib(SIG, lane & 15), ky = nib(KEY, ys);
  float4 bias1[CTW];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) bias1[ct] = *reinterpret_cast<const float4*>(a.b1 + (wt + ct) * 16 + 4 * q);
  __syncthreads();  // every wave is done reading x
  // conv1's output in place: relu(acc + b1) as bf16 at source column t + 1 (image column x0 - 1 + t)
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) {
    const int n = (wt + ct) * 16 + 4 * q;
    const float4 b4 = bias1[ct];
#pragma unroll
    for (int t = 0; t < 12; ++t) {
      const bool img = (unsigned)(x0 - 1 + t) < (unsigned)BW;
      const float v0 = fmaxf(acc[t][ct][0] + b4.x, 0.f), v1 = fmaxf(acc[t][ct][1] + b4.y, 0.f);
      const float v2 = fmaxf(acc[t][ct][2] + b4.z, 0.f), v3 = fmaxf(acc[t][ct][3] + b4.w, 0.f);
      uint2 o;
      o.x = img ? ((uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16)) : 0u;
      o.y = img ? ((uint32_t)f32_to_bf16(v2) | ((uint32_t)f32_to_bf16(v3) << 16)) : 0u;
      *reinterpret_cast<uint2*>(lds + (16 * (t + 1) + ys) * RB + (((n >> 3) ^ ky) << 4) + ((n & 7) << 1)) = o;
      acc[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  // conv2's ring fills while the barrier waits
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
    for (int i = 0; i < RDB; ++i) bq[ct][i] = wld<TNS>(wrs2, ct, band_step<NC>(i), lane);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 12; ++t)
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) asm volatile("" : "+a"(acc[t][ct]));
  band_all<C, C, 10, NSRC, 16 * RB, 12, RDB>(lds, wrs2, bq, acc, lane);
  BSTAMP(2);
  // epilogue: the residual straight into registers in the accumulator layout (this lane's image row
  // ys, 4 channels, every band column): all loads in flight before the barrier that waits for the other
  // waves' conv2, so their latency hides behind it (staged through LDS after the barrier it was a
  // serialised 32 k-cycle phase in the stamps); + b2 + residual, ReLU, bf16 to LDS, 16-B stores
  uint2 rr[CTW][10];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) {
    const int n = (wt + ct) * 16 + 4 * q;
#pragma unroll
    for (int t = 0; t < 10; ++t) rr[ct][t] = *reinterpret_cast<const uint2*>(src + (size_t)(ys * BW + x0 + t) * C + n);
  }
  float4 bias2[CTW];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) bias2[ct] = *reinterpret_cast<const float4*>(a.b2 + (wt + ct) * 16 + 4 * q);
  __syncthreads();  // conv1's output is no longer read
  BSTAMP(3);
  constexpr int ONCH = C / 8, NR = 10 * 16 * ONCH;
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) {
    const int n = (wt + ct) * 16 + 4 * q;
    const float4 b4 = bias2[ct];
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      const uint2 r = rr[ct][t];
      float v0 = acc[t][ct][0] + b4.x, v1 = acc[t][ct][1] + b4.y, v2 = acc[t][ct][2] + b4.z, v3 = acc[t][ct][3] + b4.w;
      v0 += __uint_as_float(r.x << 16); v1 += __uint_as_float(r.x & 0xffff0000u);
      v2 += __uint_as_float(r.y << 16); v3 += __uint_as_float(r.y & 0xffff0000u);
      v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      uint2 o;
      o.x = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
      o.y = (uint32_t)f32_to_bf16(v2) | ((uint32_t)f32_to_bf16(v3) << 16);
      *reinterpret_cast<uint2*>(lds + (t * 16 + ys) * RB + (((n >> 3) ^ ky) << 4) + ((n & 7) << 1)) = o;
    }
  }
  __syncthreads();
  BSTAMP(4);
  bf16_t* gout = a.out + (size_t)b * BH * BW * C;
  for (int i = tid; i < NR; i += BNT) {
    const int row = i / ONCH, ch = i % ONCH, t = row >> 4, y = row & 15;
    *reinterpret_cast<uint4*>(gout + (size_t)(y * BW + x0 + t) * C + ch * 8) =
        *reinterpret_cast<const uint4*>(lds + row * RB + ((ch ^ nib(KEY, y)) << 4));
  }
  BSTAMP(5);
  BSTAMP_REAL(7);
}

}  // namespace

static thread_local int g_band_xt = 5;  // output columns per workgroup (mzba_conv_band_set_xt; per thread)

extern "C" {

// band width (output columns per workgroup): 5 (default: two workgroups per CU, one's band staging and
// epilogue beside the other's MFMAs; B = 4096, isolated: 256->256 1247 -> 1218 us, 128->128 423 -> 378,
// 128->256 787 -> 691, profiles/r02/band_xt/) or 10 (one workgroup per CU at Cin 256)
int mzba_conv_band_set_xt(int xt) {
  if (xt != 5 && xt != 10) return -1;
  g_band_xt = xt;
  return 0;
}

// ResidualBlock(C) at 16x20 in one launch (band_res_kernel), C in {128, 256}
int mzba_conv_band_res_supported(int H, int W, int C) { return H == BH && W == BW && (C == 256 || C == 128); }

int mzba_conv_band_res(const void* in, const void* w1, const float* b1, const void* w2, const float* b2, void* out,
                       int B, int H, int W, int C, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && in && w1 && b1 && w2 && b2 && out && in != out && mzba_conv_band_res_supported(H, W, C), -1);
  BandResArgs a{(const bf16_t*)in, (const bf16_t*)w1, b1, (const bf16_t*)w2, b2, (bf16_t*)out, B};
  if (C == 256) hipLaunchKernelGGL(band_res_kernel<256>, dim3(2 * B), dim3(BNT), 0, stream, a);
  else hipLaunchKernelGGL(band_res_kernel<128>, dim3(2 * B), dim3(BNT), 0, stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

#ifdef BAND_STAMPS
int mzba_band_stamps_read(unsigned long long* host, int nrows) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mz_band_stamps), sizeof(unsigned long long) * BST_N * nrows);
}
#endif

int mzba_conv_band_supported(int H, int W, int Cin, int Cout, int ks) {
  return H == BH && W == BW && ks == 3 && ((Cin == 64 && Cout == 128) || ((Cin == 128 || Cin == 256) &&
                                                                           (Cout == 128 || Cout == 256)));
}

// 3x3 conv, stride 1, pad 1, on B images of 16x20 (NHWC bf16, env stride 320*Cin / 320*Cout):
// out = [relu](conv(in, W) + bias [+ res]); weights in the tower packing (+8 KB pad). out may not alias in.
int mzba_conv_band(const void* in, const void* wf16, const float* bias, const void* res, void* out, int B, int H,
                   int W, int Cin, int Cout, int relu, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && in && wf16 && bias && out && in != out && mzba_conv_band_supported(H, W, Cin, Cout, 3), -1);
  BandArgs a{(const bf16_t*)in, (const bf16_t*)wf16, bias, (const bf16_t*)res, (bf16_t*)out, B, relu};
  const bool narrow = g_band_xt == 5;
  dim3 grid((narrow ? 4 : 2) * B);
#define MZ_BAND(CI, CO)                                                                                   \
  do {                                                                                                     \
    if (narrow) hipLaunchKernelGGL((band_conv_kernel<CI, CO, 5>), grid, dim3(BNT), 0, stream, a);          \
    else hipLaunchKernelGGL((band_conv_kernel<CI, CO, 10>), grid, dim3(BNT), 0, stream, a);                \
  } while (0)
  if (Cin == 256 && Cout == 256) MZ_BAND(256, 256);
  else if (Cin == 128 && Cout == 256) MZ_BAND(128, 256);
  else if (Cin == 128 && Cout == 128) MZ_BAND(128, 128);
  else if (Cin == 64) MZ_BAND(64, 128);
  else MZ_BAND(256, 128);
#undef MZ_BAND
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
