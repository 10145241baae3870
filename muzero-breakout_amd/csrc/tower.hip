// Fused residual tower for the dynamics / prediction nets (bf16 or fp16, gfx950 MFMA).
//
// The towers are nblocks x ResidualBlock(256) on a 4x5 latent (src/networks.py:19-35,
// 124-131, 190-197). Launching every conv separately re-stages the activations into LDS
// and writes them back to HBM 28 times per tower. Here ONE workgroup owns E = 4 whole envs
// (80 rows) x all 256 channels for the whole tower:
//   * X (block input / output) and T (conv1 output) stay resident in LDS (2 x 40 KB) across
//     every block. LDS row of (env e, latent y, x) = 16x + 4y + e: a 16-row MFMA tile is one
//     latent COLUMN x of all 4 envs, so a 3x3 tap (dy, dx) maps tile x to tile x + dx whole
//     (tiles with x + dx outside 0..4 are skipped: 39 of 45 tile-taps run) and shifts rows
//     by 4 dy inside the tile. 16-B chunks are XOR-swizzled by (row & 15) = 4y + e; rows that
//     fall outside y = 0..3 read a 16-row zero block at the row key ((y + dy) & 3) * 4 + e,
//     so every ds_read_b128 lane group hits 16 distinct bank slots for every tap;
//   * weights stream into VGPRs from a 16-column fragment-major packing
//     wf16[col tile][k step][lane][8] with taps ordered (dx, dy) (agent.pack_tower_conv),
//     one coalesced 1 KB wave load per 32-deep k step and column tile, 4 steps in flight;
//     each of the 8 waves owns 32 output channels;
//   * v_mfma_f32_16x16x32_bf16: up to 5 row tiles x 2 column tiles per wave; MFMA /
//     next-step ds_read_b128 / VALU interleaved by sched_group_barrier;
//   * conv1 epilogue: + bias, ReLU -> T (LDS); conv2: accumulator initialised with
//     bias + residual X, ReLU -> X in place (each element is owned by one lane).
// Input is read from HBM once (optional per-env slot gather from the latent node pool) and
// the tower output written once. Grid: ceil(B / 4) workgroups of 512 threads.
#include "common.h"
#include "tree_dev.h"
#include "elt.h"  // Elt<EL> (bf16 / fp16 images and weights), unpack8

namespace {

// an MFMA B fragment shifted by 4 columns inside each 16-lane row (zeros shifted in): the same tile
// read one latent row up / down (columns = image rows 4y + e)
template <int EL> MZ_DEV typename Elt<EL>::v8 dpp_shl4(typename Elt<EL>::v8 v) {
  int4 i = __builtin_bit_cast(int4, v);
  i.x = __builtin_amdgcn_update_dpp(0, i.x, 0x104, 0xf, 0xf, true);
  i.y = __builtin_amdgcn_update_dpp(0, i.y, 0x104, 0xf, 0xf, true);
  i.z = __builtin_amdgcn_update_dpp(0, i.z, 0x104, 0xf, 0xf, true);
  i.w = __builtin_amdgcn_update_dpp(0, i.w, 0x104, 0xf, 0xf, true);
  return __builtin_bit_cast(typename Elt<EL>::v8, i);
}

constexpr int TE = 4;              // envs per workgroup
constexpr int TROWS = 80;          // TE * 20 (4x5 latent)
constexpr int TC = 256;            // channels
constexpr int TROWB = TC * 2;      // 512 B per LDS row
constexpr int TR = 5;              // 16-row tiles = latent columns x
constexpr int TNS = 9 * TC / 32;   // 72 k steps per 3x3 conv
constexpr int TD = 4;              // 4-env 8-wave kernel's weight ring depth (k steps); divides a tap's 8
static_assert(8 % TD == 0, "ring index restarts at every tap");
// tower8 weight ring depth in entries (one entry = one 1 KB fragment per column tile): two k steps of
// the one-pass k loop (3 column shifts each); a ring entry count must divide the 24 of a dy
template <int NQ> constexpr int t8d = 6;
constexpr int TNT = 512;
constexpr int IMG = TROWS * TROWB;         // one activation image (40 KB)
constexpr int LDS_X = 0, LDS_T = IMG, LDS_Z = 2 * IMG, LDS_BYTES = 2 * IMG + 16 * TROWB;

struct TowerArgs {
  const bf16_t* in;
  long long in_env_stride;
  const int32_t* slot;
  long long in_slot_stride;
  bf16_t* out;               // [B][20][256]
  const bf16_t* wf;          // per conv: [16 col tiles][72 k steps][64][8], convs back to back (+pad)
  const float* bias;         // per conv: [256]
  int nblocks;               // residual blocks (2 convs each)
  int B;
  mzba_tower_ext x;          // fused prologue / epilogue (4-env kernel); all zero = plain tower
  TreeArgs tree;             // prediction epilogue: backup(tree_sim) + select(tree_sim + 1) per env
  int tree_on, tree_sim;
  float tree_gamma;
  const float* tree_r;
};

#ifdef TOWER_STAMPS
// diagnostic build only (make tower-stamps -> libmzba_tstamp.so, tools/stamp_tower.py): s_memtime at
// the phase boundaries of every conv, per workgroup and wave; slot 2 + 6 ci + phase for conv ci
// (phase 0 k loop start, 1/2/3 after the dx = -1/0/+1 taps, 4 after the first barrier, 5 after the
// write-back barrier); 0 entry, 1 after staging, TST_N - 3/-2 s_memrealtime at entry / exit, TST_N - 1 exit
constexpr int TST_N = 192, TST_WG = 1024;
__device__ unsigned long long mz_tower_stamps[TST_WG * 4][TST_N];
MZ_DEV void tstamp(int k, bool real = false) {
  if ((threadIdx.x & 63) == 0 && blockIdx.x < TST_WG && k < TST_N)
    mz_tower_stamps[blockIdx.x * 4 + (threadIdx.x >> 6)][k] =
        real ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
}
#define TSTAMP(k) tstamp(k)
#define TSTAMP_END() (tstamp(TST_N - 2, true), tstamp(TST_N - 1))
#else
#define TSTAMP(k) \
  do {            \
  } while (0)
#define TSTAMP_END() \
  do {               \
  } while (0)
#endif

// LDS row of (env e, latent position p = 5y + x) and the byte offset of (row, 16-B chunk)
MZ_DEV int trow(int e, int p) { return (p % 5) * 16 + (p / 5) * 4 + e; }
MZ_DEV int toff(int row, int chunk) { return row * TROWB + ((chunk ^ (row & 15)) << 4); }

// 4-wave kernel geometry: NQ env quads per workgroup (2: the 8-env kernel; 1: 4 envs, every wave
// 4 column tiles of 5 row tiles — half the LDS A reads per MFMA of the 8-wave 4-env kernel)
template <int NQ>
struct T8 {
  static constexpr int E = 4 * NQ, ROWS = 80 * NQ, NRT = 5 * NQ, NT = 256, CT = 4;  // 4 waves
  static constexpr int IMG = ROWS * TROWB;                   // 40 / 80 KB
  static constexpr int LZ = IMG, BYTES = IMG + 16 * TROWB;   // + 16 zero rows
};
namespace t8 {
constexpr int NT = 256, CT = 4;
// LDS row of (env e, latent position p = 5y + x): env quad (e >> 2) owns tiles 5 (e >> 2) .. +4
MZ_DEV int row8(int e, int p) { return (e >> 2) * 80 + (p % 5) * 16 + (p / 5) * 4 + (e & 3); }
}  // namespace t8

// Image geometry of the 4-wave kernels: GROUPS groups of TX 16-row tiles; a tile is one latent
// column x of EG envs x YS latent rows (row in tile = EG * y + e); a 3x3 tap (dy, dx) maps tile x to
// tile x + dx whole and shifts rows by EG * dy; rows leaving y = 0..YS-1 read the zero block (LZ) at
// the row key ((y + dy) mod YS) * EG + e, so every ds_read_b128 lane group hits 16 distinct keys.
template <int NQ>
struct Geo45 {  // the 4x5 latent: NQ env quads, 5 tiles each (tower8_kernel)
  static constexpr int GROUPS = NQ, TX = 5, EG = 4, YS = 4, LZ = T8<NQ>::LZ;
};
struct Geo810 {  // the 8x10 latent of the representation tail: 2 envs, 10 tiles (rep_tail_kernel)
  static constexpr int GROUPS = 1, TX = 10, EG = 2, YS = 8, LZ = 160 * TROWB;
};

// A-row addressing of this lane for latent row shift dy: byte offset of its row in source
// tile 0 (or of its zero-block row), the per-tile stride (0 for zero rows) and the swizzle key
MZ_DEV void tap_rows(int srcimg, int y, int e, int dy, int& base, int& tstride, int& sw, int zblk = LDS_Z) {
  const int yy = y + dy;
  const bool ok = (unsigned)yy < 4u;
  const int key = ((yy & 3) << 2) | e;
  base = ok ? srcimg + key * TROWB : zblk + key * TROWB;
  tstride = ok ? 16 * TROWB : 0;
  sw = key << 4;
}

// the 24 k steps (3 dy x 8 channel chunks) of the taps with column shift DX
template <int EL, int DX>
__device__ __forceinline__ void tower_dx(const uint8_t* __restrict__ lds, int srcimg, const uint4* __restrict__ wp0,
                                         const uint4* __restrict__ wp1, uint4 (&b0q)[TD], uint4 (&b1q)[TD],
                                         f32x4 (&acc0)[TR], f32x4 (&acc1)[TR], int lane) {
  constexpr int NT = DX == 0 ? 5 : 4;   // active tiles
  constexpr int A0 = DX < 0 ? 1 : 0;    // first accumulator tile (output column x)
  constexpr int S0 = DX > 0 ? 1 : 0;    // first source tile (x + dx)
  constexpr int SB = (DX + 1) * 24;     // first k step of this column shift
  const int q = lane >> 4, y = (lane & 15) >> 2, e = lane & 3;
  int base, tst, sw;
  tap_rows(srcimg + S0 * 16 * TROWB, y, e, -1, base, tst, sw);
  typename Elt<EL>::v8 afc[NT], afn[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) afc[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + base + j * tst + ((q << 4) ^ sw));
  constexpr int NC = TC / 32;  // 8 k steps per tap
#pragma unroll 1
  for (int dyi = 0; dyi < 3; ++dyi) {
    int nbase, ntst, nsw;
    tap_rows(srcimg + S0 * 16 * TROWB, y, e, dyi < 2 ? dyi : 1, nbase, ntst, nsw);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int s = SB + dyi * NC + c;
      const typename Elt<EL>::v8 w0 = __builtin_bit_cast(typename Elt<EL>::v8, b0q[c % TD]);
      const typename Elt<EL>::v8 w1 = __builtin_bit_cast(typename Elt<EL>::v8, b1q[c % TD]);
      b0q[c % TD] = wp0[(size_t)(s + TD) * 64];
      b1q[c % TD] = wp1[(size_t)(s + TD) * 64];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc0[A0 + j] = Elt<EL>::mfma(w0, afc[j], acc0[A0 + j]);
        acc1[A0 + j] = Elt<EL>::mfma(w1, afc[j], acc1[A0 + j]);
        if (c + 1 < NC)
          afn[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + base + j * tst + (((4 * (c + 1) + q) << 4) ^ sw));
        else
          afn[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + nbase + j * ntst + ((q << 4) ^ nsw));
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NT; ++j) afc[j] = afn[j];
    }
    base = nbase; tst = ntst; sw = nsw;
  }
}

// the 8 k steps of a 1x1 conv (centre tap only: every row valid, all 5 tiles)
template <int EL>
__device__ __forceinline__ void tower_center(const uint8_t* __restrict__ lds, int srcimg, const uint4* __restrict__ wp0,
                                             const uint4* __restrict__ wp1, uint4 (&b0q)[TD], uint4 (&b1q)[TD],
                                             f32x4 (&acc0)[TR], f32x4 (&acc1)[TR], int lane) {
  const int q = lane >> 4, key = lane & 15;
  const int base = srcimg + key * TROWB, sw = key << 4;
  typename Elt<EL>::v8 afc[TR], afn[TR];
#pragma unroll
  for (int j = 0; j < TR; ++j) afc[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + base + j * 16 * TROWB + ((q << 4) ^ sw));
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const typename Elt<EL>::v8 w0 = __builtin_bit_cast(typename Elt<EL>::v8, b0q[c % TD]);
    const typename Elt<EL>::v8 w1 = __builtin_bit_cast(typename Elt<EL>::v8, b1q[c % TD]);
    if (c + TD < 8) {
      b0q[c % TD] = wp0[(size_t)(c + TD) * 64];
      b1q[c % TD] = wp1[(size_t)(c + TD) * 64];
    }
#pragma unroll
    for (int j = 0; j < TR; ++j) {
      acc0[j] = Elt<EL>::mfma(w0, afc[j], acc0[j]);
      acc1[j] = Elt<EL>::mfma(w1, afc[j], acc1[j]);
      if (c + 1 < 8)
        afn[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + base + j * 16 * TROWB + (((4 * (c + 1) + q) << 4) ^ sw));
    }
#pragma unroll
    for (int j = 0; j < TR; ++j) afc[j] = afn[j];
  }
}

// One conv of the 4-env kernel, this wave's two 16-channel column tiles ct0, ct0 + 1 of a weight pack
// with `tns` k steps per tile (72: 3x3, 8: 1x1); pack column n lands on image channel nout + n.
// MODE 0: bias; 1: bias + residual (the destination image); 2: bias + act_bias[pos][act[e]][n].
// Epilogue: ReLU -> bf16 -> dst.
template <int EL, int MODE, bool CENTER>
__device__ __forceinline__ void tower_conv(uint8_t* __restrict__ lds, int srcimg, int dstimg,
                                           const uint4* __restrict__ wconv, int tns, int ct0,
                                           const float* __restrict__ bconv, int nout,
                                           const float* __restrict__ actb, const int* acts, int A, int lane) {
  const int q = lane >> 4, l16 = lane & 15;
  const int ct1 = ct0 + 1;
  const uint4* wp0 = wconv + (size_t)ct0 * tns * 64 + lane;
  const uint4* wp1 = wconv + (size_t)ct1 * tns * 64 + lane;
  uint4 b0q[TD], b1q[TD];
#pragma unroll
  for (int i = 0; i < TD; ++i) { b0q[i] = wp0[(size_t)i * 64]; b1q[i] = wp1[(size_t)i * 64]; }
  // weights are the MFMA A operand: D[pack channel 16 ct + 4q + i][row 16 rt + l16], so a lane
  // holds 4 consecutive channels of one row (8-byte LDS reads / writes); row l16 of tile rt =
  // latent (y = l16 >> 2, x = rt) of env l16 & 3
  const int n0 = ct0 * 16 + 4 * q, n1 = ct1 * 16 + 4 * q;  // pack channels
  const int c0 = nout + n0, c1 = nout + n1;                // image channels
  const float4 bb0 = *reinterpret_cast<const float4*>(bconv + n0);
  const float4 bb1 = *reinterpret_cast<const float4*>(bconv + n1);
  f32x4 acc0[TR], acc1[TR];
#pragma unroll
  for (int rt = 0; rt < TR; ++rt) {
    f32x4 r0 = {bb0.x, bb0.y, bb0.z, bb0.w}, r1 = {bb1.x, bb1.y, bb1.z, bb1.w};
    const int row = rt * 16 + l16;
    if (MODE == 1) {
      const uint2 x0 = *reinterpret_cast<const uint2*>(lds + dstimg + toff(row, c0 >> 3) + ((c0 & 7) << 1));
      const uint2 x1 = *reinterpret_cast<const uint2*>(lds + dstimg + toff(row, c1 >> 3) + ((c1 & 7) << 1));
      r0[0] += Elt<EL>::lo(x0.x); r0[1] += Elt<EL>::hi(x0.x);
      r0[2] += Elt<EL>::lo(x0.y); r0[3] += Elt<EL>::hi(x0.y);
      r1[0] += Elt<EL>::lo(x1.x); r1[1] += Elt<EL>::hi(x1.x);
      r1[2] += Elt<EL>::lo(x1.y); r1[3] += Elt<EL>::hi(x1.y);
    } else if (MODE == 2) {
      const float* t = actb + ((size_t)((l16 >> 2) * 5 + rt) * A + acts[l16 & 3]) * TC;
      const float4 t0 = *reinterpret_cast<const float4*>(t + n0), t1 = *reinterpret_cast<const float4*>(t + n1);
      r0[0] += t0.x; r0[1] += t0.y; r0[2] += t0.z; r0[3] += t0.w;
      r1[0] += t1.x; r1[1] += t1.y; r1[2] += t1.z; r1[3] += t1.w;
    }
    acc0[rt] = r0;
    acc1[rt] = r1;
  }
  if (CENTER) {
    tower_center<EL>(lds, srcimg, wp0, wp1, b0q, b1q, acc0, acc1, lane);
  } else {
    tower_dx<EL, -1>(lds, srcimg, wp0, wp1, b0q, b1q, acc0, acc1, lane);
    tower_dx<EL, 0>(lds, srcimg, wp0, wp1, b0q, b1q, acc0, acc1, lane);
    tower_dx<EL, 1>(lds, srcimg, wp0, wp1, b0q, b1q, acc0, acc1, lane);
  }
#pragma unroll
  for (int rt = 0; rt < TR; ++rt) {
    const int row = rt * 16 + l16;
    uint2 o0, o1;
    o0.x = Elt<EL>::pack2(fmaxf(acc0[rt][0], 0.f), fmaxf(acc0[rt][1], 0.f));
    o0.y = Elt<EL>::pack2(fmaxf(acc0[rt][2], 0.f), fmaxf(acc0[rt][3], 0.f));
    o1.x = Elt<EL>::pack2(fmaxf(acc1[rt][0], 0.f), fmaxf(acc1[rt][1], 0.f));
    o1.y = Elt<EL>::pack2(fmaxf(acc1[rt][2], 0.f), fmaxf(acc1[rt][3], 0.f));
    *reinterpret_cast<uint2*>(lds + dstimg + toff(row, c0 >> 3) + ((c0 & 7) << 1)) = o0;
    *reinterpret_cast<uint2*>(lds + dstimg + toff(row, c1 >> 3) + ((c1 & 7) << 1)) = o1;
  }
}

// Linear heads on an LDS image (networks.py:147, 207, 221): head h reads image channels
// [hc0[h], hc0[h] + hC[h]) of the 20 positions of each env, K = 20 hC[h] in (position, channel)
// order against bf16 weights lw[h][16][K]. One v_mfma_f32_16x16x32_bf16 per 32-deep k step
// (A rows = the 4 envs, zero-padded to 16; B cols = outputs), k steps split over the 8 waves,
// partial sums added through LDS in wave order; then softmax (dec_kind 0) or support decode (1).
template <int EL, int NE, int NW, bool R8>
__device__ __forceinline__ void tower_heads(const TowerArgs& a, const uint8_t* __restrict__ lds, int img,
                                            int nh, const int (&hc0)[2], const int (&hC)[2], const int (&kind)[2],
                                            float* part, float* lg, float (*dec)[8][4], int env0, int nenv,
                                            int tid) {
  // NE envs per workgroup, NW waves; part: [NW][8][16] partial sums, lg: [2][8][16] logits
  const int lane = tid & 63, wave = tid >> 6, q = lane >> 4, el = lane & 15;
  for (int hd = 0; hd < nh; ++hd) {
    const int C = hC[hd], K = 20 * C, nk = K / 32;
    const bf16_t* wr = reinterpret_cast<const bf16_t*>(a.x.lw[hd]) + (size_t)el * K;
    const int er = el < nenv ? el : 0;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    // the wave's k steps s = wave + NW u in batches of HU: every weight load of a batch in flight
    // before its first MFMA (one loop iteration per k step waited one L2 round trip each: 20-40
    // per head and wave), MFMAs in the same order as before
    constexpr int HU = 10;
    for (int s0 = wave; s0 < nk; s0 += NW * HU) {
      typename Elt<EL>::v8 bv[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int s = min(s0 + u * NW, nk - 1);
        bv[u] = *reinterpret_cast<const typename Elt<EL>::v8*>(wr + s * 32 + q * 8);
      }
      auto kstep = [&](int u) {
        const int k = (s0 + u * NW) * 32 + q * 8;
        const int pos = k / C, c = hc0[hd] + (k - pos * C);
        const int row = R8 ? t8::row8(er, pos) : trow(er, pos);
        typename Elt<EL>::v8 av = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + img + toff(row, c >> 3));
        if (el >= NE) av = typename Elt<EL>::v8{};
        acc = Elt<EL>::mfma(av, bv[u], acc);
      };
      if (s0 + (HU - 1) * NW < nk) {  // whole batch (always, for K = 20 x 128 / 256 and NW = 4 / 8)
#pragma unroll
        for (int u = 0; u < HU; ++u) kstep(u);
      } else {
#pragma unroll
        for (int u = 0; u < HU; ++u)
          if (s0 + u * NW < nk) kstep(u);
      }
    }
    if (4 * q < NE)  // D[row = env 4q + i][col = output el]
#pragma unroll
      for (int i = 0; i < 4; ++i) part[(wave * 8 + 4 * q + i) * 16 + el] = acc[i];
    __syncthreads();
    if (tid < NE * 16) {
      const int e = tid >> 4, o = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v = v + part[(w * 8 + e) * 16 + o];
      if (o < a.x.lO[hd]) lg[(hd * 8 + e) * 16 + o] = v + a.x.lb[hd][o];
    }
    __syncthreads();
  }
  if (tid < NE * nh) {
    const int hd = tid / NE, e = tid % NE, b = env0 + e;
    if (e < nenv) {
      const int O = a.x.lO[hd];
      float l[16];
      for (int o = 0; o < O; ++o) {
        l[o] = lg[(hd * 8 + e) * 16 + o];
        if (a.x.logits[hd]) a.x.logits[hd][(size_t)b * O + o] = l[o];
      }
      if (kind[hd] == 0) {
        float m = l[0];
        for (int o = 1; o < O; ++o) m = fmaxf(m, l[o]);
        float ex[16], sum = 0.f;
        for (int o = 0; o < O; ++o) { ex[o] = expf(l[o] - m); sum = sum + ex[o]; }
        for (int o = 0; o < O; ++o) {
          const float p = ex[o] / sum;
          a.x.dec[hd][(size_t)b * O + o] = p;
          if (o < 4) dec[hd][e][o] = p;
        }
      } else {
        const float d = decode_support(l, O, a.x.smin, a.x.smax);
        a.x.dec[hd][b] = d;
        dec[hd][e][0] = d;
      }
    }
  }
}

// _scale_state (networks.py:314-328) of the tower output X: per env (h - min) / (max - min + 1e-8)
// in f32, bf16 result to out (and to the pool slot). 128 threads per env, 5 chunks each.
template <int EL>
__device__ __forceinline__ void tower_scale(const TowerArgs& a, const uint8_t* __restrict__ lds, float (*mm)[2][2],
                                            int env0, int nenv, int tid) {
  const int e = tid >> 7, t = tid & 127;
  uint4 v[5];
  float mn = INFINITY, mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int i = u * 128 + t, p = i >> 5, c = i & 31;
    v[u] = *reinterpret_cast<const uint4*>(lds + LDS_X + toff(trow(e, p), c));
    float f[8];
    unpack8<EL>(v[u], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) { mn = fminf(mn, f[j]); mx = fmaxf(mx, f[j]); }
  }
  for (int o = 32; o > 0; o >>= 1) { mn = fminf(mn, __shfl_xor(mn, o)); mx = fmaxf(mx, __shfl_xor(mx, o)); }
  if ((t & 63) == 0) { mm[e][t >> 6][0] = mn; mm[e][t >> 6][1] = mx; }
  __syncthreads();
  mn = fminf(mm[e][0][0], mm[e][1][0]);
  mx = fmaxf(mm[e][0][1], mm[e][1][1]);
  if (e >= nenv) return;
  const float den = (mx - mn) + 1e-8f;
  const int b = env0 + e;
  bf16_t* o1 = a.out ? a.out + (size_t)b * 20 * TC : nullptr;  // null: the node-pool slot only
  bf16_t* o2 = a.x.pool ? reinterpret_cast<bf16_t*>(a.x.pool) + (size_t)b * a.x.pool_env_stride +
                              (size_t)a.x.pool_slot * 20 * TC
                        : nullptr;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int i = u * 128 + t, p = i >> 5, c = i & 31;
    float f[8];
    unpack8<EL>(v[u], f);
    const uint4 r = make_uint4(pack_bf16x2((f[0] - mn) / den, (f[1] - mn) / den), pack_bf16x2((f[2] - mn) / den, (f[3] - mn) / den),
                               pack_bf16x2((f[4] - mn) / den, (f[5] - mn) / den), pack_bf16x2((f[6] - mn) / den, (f[7] - mn) / den));
    if (o1) *reinterpret_cast<uint4*>(o1 + p * TC + c * 8) = r;
    if (o2) *reinterpret_cast<uint4*>(o2 + p * TC + c * 8) = r;
  }
}

template <int EL>
__global__ __launch_bounds__(TNT, 2) void tower_kernel(TowerArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];  // X | T | 16 zero rows
  __shared__ long long envoff[TE];
  __shared__ int acts[TE];
  __shared__ float part[8 * 8 * 16];  // head partial sums [wave][env][output]; min/max scratch
  __shared__ float lg[2 * 8 * 16];    // head logits [head][env][output]
  __shared__ float dec[2][8][4];      // decoded head outputs [head][env][output]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int env0 = blockIdx.x * TE;
  const int nenv = min(TE, a.B - env0);
  const int rows = nenv * 20;
  const bool pro = a.x.w0 != nullptr;
  if (tid < TE) {
    const int b = env0 + (tid < nenv ? tid : 0);
    long long off = (long long)b * a.in_env_stride;
    if (a.slot) off += (long long)a.slot[b] * a.in_slot_stride;
    envoff[tid] = off;
    acts[tid] = pro ? a.x.act[b] : 0;
  }
  __syncthreads();
  // stage X (80 rows x 32 chunks = 2560 chunks, 5 per thread; into T when a prologue conv follows)
  // and zero the zero block
  {
    const int stg = pro ? LDS_T : LDS_X;
    uint4 v[5];
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int i = u * TNT + tid;
      const int r = i >> 5, c = i & 31;
      const bool ok = r < rows;
      const int rr = ok ? r : 0;
      v[u] = Elt<EL>::from_bf16(*reinterpret_cast<const uint4*>(a.in + envoff[rr / 20] + (long long)(rr % 20) * TC + c * 8));
      if (!ok) v[u] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int i = u * TNT + tid;
      const int r = i >> 5;
      *reinterpret_cast<uint4*>(lds + stg + toff(trow(r / 20, r % 20), i & 31)) = v[u];
    }
    *reinterpret_cast<uint4*>(lds + LDS_Z + tid * 16) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  if (pro) {  // dynamics ConvBlock: T -> X
    tower_conv<EL, 2, false>(lds, LDS_T, LDS_X, reinterpret_cast<const uint4*>(a.x.w0), TNS, 2 * wave, a.x.b0, 0,
                         a.x.act_bias, acts, a.x.A, lane);
    __syncthreads();
  }
  const uint4* wf = reinterpret_cast<const uint4*>(a.wf);
  constexpr size_t WCONV = (size_t)16 * TNS * 64;  // uint4 per conv
  for (int blk = 0; blk < a.nblocks; ++blk) {
    tower_conv<EL, 0, false>(lds, LDS_X, LDS_T, wf + (2 * blk) * WCONV, TNS, 2 * wave, a.bias + (2 * blk) * TC, 0,
                         nullptr, nullptr, 0, lane);
    __syncthreads();
    tower_conv<EL, 1, false>(lds, LDS_T, LDS_X, wf + (2 * blk + 1) * WCONV, TNS, 2 * wave,
                         a.bias + (2 * blk + 1) * TC, 0, nullptr, nullptr, 0, lane);
    __syncthreads();
  }
  if (a.x.epilogue == 1) {  // dynamics: reward ConvBlock1x1 (X -> T), Linear + decode, scaled latent
    tower_conv<EL, 0, true>(lds, LDS_X, LDS_T, reinterpret_cast<const uint4*>(a.x.we1), 8, 2 * wave, a.x.be1, 0,
                        nullptr, nullptr, 0, lane);
    __syncthreads();
    const int hc0[2] = {0, 0}, hC[2] = {TC, 0}, kind[2] = {1, 0};
    tower_heads<EL, TE, 8, false>(a, lds, LDS_T, 1, hc0, hC, kind, part, lg, dec, env0, nenv, tid);
    tower_scale<EL>(a, lds, reinterpret_cast<float(*)[2][2]>(part), env0, nenv, tid);
    return;
  }
  if (a.x.epilogue == 2) {  // prediction: policy 3x3 -> T[0,128), value 1x1 -> T[128,256); Linears
    if (wave < 4)
      tower_conv<EL, 0, false>(lds, LDS_X, LDS_T, reinterpret_cast<const uint4*>(a.x.we3), TNS, 2 * wave, a.x.be3, 0,
                           nullptr, nullptr, 0, lane);
    else
      tower_conv<EL, 0, true>(lds, LDS_X, LDS_T, reinterpret_cast<const uint4*>(a.x.we1), 8, 2 * (wave - 4), a.x.be1,
                          128, nullptr, nullptr, 0, lane);
    __syncthreads();
    const int hc0[2] = {0, 128}, hC[2] = {128, 128}, kind[2] = {0, 1};
    tower_heads<EL, TE, 8, false>(a, lds, LDS_T, 2, hc0, hC, kind, part, lg, dec, env0, nenv, tid);
    if (a.tree_on) {  // this simulation's backup and the next selection (mcts.py:136-234), per env
      __syncthreads();
      if (tid < nenv) {
        const int b = env0 + tid;
        tree_backup_env(a.tree, a.tree_sim, b, a.tree_r[b], dec[1][tid][0], &dec[0][tid][0], a.tree_gamma);
        if (a.tree_sim + 1 < a.tree.S) tree_select_env(a.tree, a.tree_sim + 1, b);
      }
    }
    return;
  }
  // write the tower output (16-B chunks, rows < rows)
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int i = u * TNT + tid;
    const int r = i >> 5, c = i & 31;
    if (r < rows)
      *reinterpret_cast<uint4*>(a.out + (long long)(env0 + r / 20) * 20 * TC + (r % 20) * TC + c * 8) =
          Elt<EL>::to_bf16(*reinterpret_cast<const uint4*>(lds + LDS_X + toff(trow(r / 20, r % 20), c)));
  }
}

// ---------------------------------------------------------------------------------------------
// 8-env variant (tower8_kernel): ONE workgroup = 8 envs (160 rows) x 256 channels, 4 waves (one per
// SIMD, up to 512 registers each), every wave all 10 row tiles x 4 column tiles (64 channels).
// Each weight fragment loaded from L2 now feeds 10 MFMAs instead of 5, halving the per-CU weight
// stream per env (the bound of the 4-env kernel). Weights are the MFMA A operand, so a
// lane's accumulator holds 4 consecutive channels of one row: 8-byte LDS epilogue stores/loads.
// One activation image: a conv reads it whole, then (after a barrier) its output overwrites it in
// place; conv1 first lifts the block input at its own output positions into registers (the residual).

// ReLU of two packed bf16 / fp16 values: the sign bit is the int16 sign, so max(i16, 0) zeroes
// negatives (and -0). relu(round(x)) == round(relu(x)) for round-to-nearest, so this equals the
// f32 ReLU before the conversion, bit for bit (one v_pk_max_i16 instead of two v_max_f32).
MZ_DEV uint32_t relu_pk(uint32_t u) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(u));
  return r;
}

// A wave's view of a weight pack: the pack, its k steps per column tile and the wave's first column
// tile. Everything but the lane's 16-B offset is wave-uniform, so the loads address off SGPRs.
struct WNext {
  __amdgpu_buffer_rsrc_t rs;  // buffer resource over the pack at the wave's first column tile
  int tstride;                // bytes per column tile (k steps x 1 KB)
  int s0;                     // nonzero: a 3x3 pack (ring entries in the order below); 0: a 1x1 pack
  // 16-B fragment of k step `step` of the wave's column tile + ct, this lane: buffer load with the
  // lane's offset in one VGPR and the (ct, step) offset in an SGPR
  MZ_DEV uint4 ld(int ct, int step, int lane) const {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, ct * tstride + step * 1024, 0));
  }
  // the same for a 3x3 pack (72 k steps per tile)
  MZ_DEV uint4 ld3(int ct, int step, int lane) const {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, ct * (TNS * 1024) + step * 1024, 0));
  }
};
MZ_DEV WNext wnext(const void* w, int tns, int ct0) {
  const uint4* p = reinterpret_cast<const uint4*>(w) + (size_t)ct0 * tns * 64;
  return WNext{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(p), 0, 0x7fffffff, 0x00020000), tns * 1024,
               tns == TNS ? 24 : 0};
}
// pack step of ring entry n (< ring depth) of a conv: 3x3 packs walk the three column shifts of each
// (dy, channel step) together (steps 0, 24, 48, 1, 25, 49, ...), 1x1 packs their steps in order
MZ_DEV int t8_first(const WNext& p, int n) { return p.s0 ? 24 * (n % 3) + n / 3 : n; }

// Weight ring of one wave: its CT column tiles x RD entries in flight (bq). A 3x3 conv walks its 72
// pack k steps (dx, dy, channel step) as 24 k-loop steps (dy, channel step) of 3 entries each, one per
// column shift: pack steps 0, 24, 48, 1, 25, 49, ... The ring runs across conv boundaries: the last RD
// entries of a 3x3 conv fetch the NEXT conv's first entries (`nxt`, t8_first), so those loads fly
// through the epilogue and both barriers (a workgroup barrier waits for LDS, not for vmcnt) and the
// next conv's first MFMAs find their weights in registers.

// A-row addressing of lane (y, e) for latent row shift dy over a whole image (every tile a source):
// byte offset of its row in tile 0 (or of its zero-block row), the per-tile stride (0 for zero rows)
// and the swizzle key
template <class G>
MZ_DEV void t8_rows(int y, int e, int dy, int& b, int& ts, int& w) {
  const int yy = y + dy;
  const bool ok = (unsigned)yy < (unsigned)G::YS;
  const int key = (yy & (G::YS - 1)) * G::EG + e;
  b = ok ? key * TROWB : G::LZ + key * TROWB;
  ts = ok ? 16 * TROWB : 0;
  w = key << 4;
}

// One k-loop pass over all three column shifts: per (dy, channel step) every tile is read from LDS
// once and feeds dx = 0 (output x), dx = -1 (output x + 1) and dx = +1 (output x - 1) within its
// group; 24 k steps per conv (three loops, one per shift, took 72 steps and 624 A reads per conv)
template <int EL, int NQ, int CT = t8::CT, class G = Geo45<NQ>>
__device__ __forceinline__ void tower8_dall(const uint8_t* __restrict__ lds, const WNext& cur, const WNext& nxt,
                                            uint4 (&bq)[CT][t8d<NQ>], f32x4 (&acc)[T8<NQ>::NRT][CT], int lane) {
  constexpr int RD = t8d<NQ>;
  constexpr int TX = G::TX, NA = G::GROUPS * TX, NC = TC / 32;
  constexpr int NM = G::GROUPS * (3 * TX - 2) * CT;  // MFMAs per step
  static_assert(RD % 3 == 0 && NM / CT >= NA, "ring triples, schedule groups");
  const int q = lane >> 4, y = (lane & 15) / G::EG, e = lane & (G::EG - 1);
  int base, tst, sw;
  t8_rows<G>(y, e, -1, base, tst, sw);
  typename Elt<EL>::v8 afc[NA], afn[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) afc[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + base + j * tst + ((q << 4) ^ sw));
#pragma unroll 1
  for (int dyi = 0; dyi < 3; ++dyi) {
    int nbase, ntst, nsw;
    t8_rows<G>(y, e, dyi < 2 ? dyi : 1, nbase, ntst, nsw);
    const bool last = dyi == 2;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      // column-tile major: the MFMAs of column tile ct (dx = 0 over all tiles, then dx = -1, dx = +1),
      // then that tile's three ring slots are reloaded with the entries of the step after next (their
      // registers are free once its MFMAs have issued: no copies, a ring of two steps in the same
      // registers); the next step's A reads ride in the first column tile's MFMA slots
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        typename Elt<EL>::v8 w[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) w[d] = __builtin_bit_cast(typename Elt<EL>::v8, bq[ct][(3 * c + d) % RD]);
#pragma unroll
        for (int j = 0; j < NA; ++j) {
          acc[j][ct] = Elt<EL>::mfma(w[1], afc[j], acc[j][ct]);
          if (ct == 0) {
            if (c + 1 < NC)
              afn[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + base + j * tst + (((4 * (c + 1) + q) << 4) ^ sw));
            else
              afn[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + nbase + j * ntst + ((q << 4) ^ nsw));
          }
        }
#pragma unroll
        for (int j = 0; j < NA; ++j)
          if (j % TX + 1 < TX) acc[j + 1][ct] = Elt<EL>::mfma(w[0], afc[j], acc[j + 1][ct]);
#pragma unroll
        for (int j = 0; j < NA; ++j)
          if (j % TX >= 1) acc[j - 1][ct] = Elt<EL>::mfma(w[2], afc[j], acc[j - 1][ct]);
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          // entry 3 (dyi * 8 + c) + d + RD: pack step 24 d + dyi * 8 + c + RD / 3, or at dy = +1 past
          // the conv's end the next conv's entry nn = 3 c + d + RD - 24
          int so = ct * (TNS * 1024) + (24 * d + dyi * NC + c + RD / 3) * 1024;
          __amdgpu_buffer_rsrc_t rs = cur.rs;
          if (3 * c + d + RD >= 3 * NC) {
            const int nn = 3 * c + d + RD - 3 * NC;
            so = last ? ct * nxt.tstride + t8_first(nxt, nn) * 1024 : so;
            rs = last ? nxt.rs : cur.rs;
          }
          bq[ct][(3 * c + d) % RD] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, so, 0));
        }
        if (ct == 0) {
#pragma unroll
          for (int j = 0; j < NA; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, NM / CT - NA, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, NM / CT, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NA; ++j) afc[j] = afn[j];
    }
    base = nbase; tst = ntst; sw = nsw;
  }
}

// the 8 k steps of a 1x1 conv on the 8-env image (centre tap: all 10 tiles, every row valid); always
// the last conv of a launch, so the ring is not continued
template <int EL, int NQ, int CT = t8::CT>
__device__ __forceinline__ void tower8_center(const uint8_t* __restrict__ lds, const WNext& cur,
                                              uint4 (&bq)[CT][t8d<NQ>], f32x4 (&acc)[T8<NQ>::NRT][CT], int lane) {
  constexpr int RD = t8d<NQ>;
  const int q = lane >> 4, key = lane & 15;
  const int base = key * TROWB, sw = key << 4;
  typename Elt<EL>::v8 afc[T8<NQ>::NRT], afn[T8<NQ>::NRT];
#pragma unroll
  for (int j = 0; j < T8<NQ>::NRT; ++j) afc[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + base + j * 16 * TROWB + ((q << 4) ^ sw));
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    typename Elt<EL>::v8 w[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      w[ct] = __builtin_bit_cast(typename Elt<EL>::v8, bq[ct][c % RD]);
      if (c + RD < 8) bq[ct][c % RD] = cur.ld(ct, c + RD, lane);
    }
#pragma unroll
    for (int j = 0; j < T8<NQ>::NRT; ++j) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        acc[j][ct] = Elt<EL>::mfma(w[ct], afc[j], acc[j][ct]);
      if (c + 1 < 8)
        afn[j] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + base + j * 16 * TROWB + (((4 * (c + 1) + q) << 4) ^ sw));
    }
#pragma unroll
    for (int j = 0; j < T8<NQ>::NRT; ++j) afc[j] = afn[j];
  }
}

// the first ring entries of a pack (the kernel's first conv; later convs are fetched by their
// predecessor)
template <int CT, int NQ>
MZ_DEV void tower8_preload(uint4 (&bq)[CT][t8d<NQ>], const WNext& p, int lane) {
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int i = 0; i < t8d<NQ>; ++i) bq[ct][i] = p.ld(ct, t8_first(p, i), lane);
}

// k loop of one conv over the 8-env image: this wave's 4 channel tiles cur.ct0..+3 of a weight pack
// with cur.tns k steps per tile (72: 3x3, 8: 1x1), weights already in the ring; a 3x3 conv leaves the
// ring holding `nxt`'s first k steps. D[pack channel 16 ct + 4q + i][row 16 rt + l16].
// MODE 0: acc starts at bias; 1: bias + res (registers); 2: bias + act_bias[pos][act[env]].
// bconv: the conv's bias (LDS for the tower convs, global for the prologue / epilogue convs).
template <int EL, int NQ, int MODE, bool CENTER, int CT = t8::CT, class G = Geo45<NQ>>
__device__ __forceinline__ void tower8_acc(const uint8_t* __restrict__ lds, const WNext& cur, const WNext& nxt,
                                           int ct0, const float* __restrict__ bconv, const float* __restrict__ actb,
                                           const int* acts, int A, const uint2 (&res)[T8<NQ>::NRT][t8::CT],
                                           uint4 (&bq)[CT][t8d<NQ>], f32x4 (&acc)[T8<NQ>::NRT][CT], int lane,
                                           int ci = 0) {
  const int q = lane >> 4, l16 = lane & 15;
  TSTAMP(2 + 6 * ci);
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = (ct0 + ct) * 16 + 4 * q;
    const float4 b4 = *reinterpret_cast<const float4*>(bconv + n);
#pragma unroll
    for (int rt = 0; rt < T8<NQ>::NRT; ++rt) {
      f32x4 v = {b4.x, b4.y, b4.z, b4.w};
      if (MODE == 1) {
        const uint2 r = res[rt][ct];
        v[0] += Elt<EL>::lo(r.x); v[1] += Elt<EL>::hi(r.x);
        v[2] += Elt<EL>::lo(r.y); v[3] += Elt<EL>::hi(r.y);
      } else if (MODE == 2) {  // row -> env quad rt / 5, latent x = rt % 5, y = l16 >> 2, env l16 & 3
        const int env = (rt / 5) * 4 + (l16 & 3), pos = (l16 >> 2) * 5 + rt % 5;
        const float4 t = *reinterpret_cast<const float4*>(actb + ((size_t)pos * A + acts[env]) * TC + n);
        v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
      }
      acc[rt][ct] = v;
    }
  }
  // the initialised accumulators pinned to AGPRs before the k loops: left to the register
  // allocator, the init values stayed in VGPRs and the dx = -1 / 0 loops of the tower convs copied
  // 44-184 accumulator registers between the files on every dy iteration (v_accvgpr_read/write,
  // up to 0.7 extra VALU per MFMA); with the pin every k loop is copy-free
#pragma unroll
  for (int rt = 0; rt < T8<NQ>::NRT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) asm volatile("" : "+a"(acc[rt][ct]));
  if (CENTER) {
    tower8_center<EL, NQ, CT>(lds, cur, bq, acc, lane);
  } else {
    TSTAMP(3 + 6 * ci);
    TSTAMP(4 + 6 * ci);
    tower8_dall<EL, NQ, CT, G>(lds, cur, nxt, bq, acc, lane);
  }
  TSTAMP(5 + 6 * ci);
}

// ReLU -> bf16 -> the image at channel nout + 16 (ct0 + ct) + 4q (8-byte stores, in place after a
// barrier); SAVE: first lift the image's values there into res (the block input = conv2's residual)
template <int EL, int NQ, bool SAVE, int CT = t8::CT>
__device__ __forceinline__ void tower8_writeback(uint8_t* __restrict__ lds, const f32x4 (&acc)[T8<NQ>::NRT][CT],
                                                 uint2 (&res)[T8<NQ>::NRT][t8::CT], int nout, int ct0, int lane) {
  const int q = lane >> 4, l16 = lane & 15;
  // row rt * 16 + l16 has swizzle key l16 for every rt: the lane's byte offset per column tile is
  // computed once, the row tile is an immediate (toff per element re-derived it, 5 VALU per store)
  int cofs[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = nout + (ct0 + ct) * 16 + 4 * q;
    cofs[ct] = l16 * TROWB + (((n >> 3) ^ l16) << 4) + ((n & 7) << 1);
  }
#pragma unroll
  for (int rt = 0; rt < T8<NQ>::NRT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      uint2* p = reinterpret_cast<uint2*>(lds + rt * 16 * TROWB + cofs[ct]);
      if (SAVE) res[rt][ct] = *p;
      uint2 o;
      o.x = relu_pk(Elt<EL>::pack2(acc[rt][ct][0], acc[rt][ct][1]));
      o.y = relu_pk(Elt<EL>::pack2(acc[rt][ct][2], acc[rt][ct][3]));
      *p = o;
    }
}

// _scale_state over the 8-env image: 32 threads per env, 20 chunks each; bf16 to out (+ pool slot)
template <int EL, int NQ>
__device__ __forceinline__ void tower8_scale(const TowerArgs& a, const uint8_t* __restrict__ lds, int env0, int nenv,
                                             int tid) {
  constexpr int TPE = t8::NT / T8<NQ>::E;  // threads per env (32 or 64), one wave holds whole envs
  const int e = tid / TPE, t = tid % TPE;
  float mn = INFINITY, mx = -INFINITY;
  for (int u = 0; u < 640 / TPE; ++u) {
    const int i = u * TPE + t, p = i >> 5, c = i & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(lds + toff(t8::row8(e, p), c));
    float f[8];
    unpack8<EL>(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) { mn = fminf(mn, f[j]); mx = fmaxf(mx, f[j]); }
  }
  for (int o = TPE / 2; o > 0; o >>= 1) { mn = fminf(mn, __shfl_xor(mn, o)); mx = fmaxf(mx, __shfl_xor(mx, o)); }
  if (e >= nenv) return;
  const float den = (mx - mn) + 1e-8f;
  const int b = env0 + e;
  bf16_t* o1 = a.out ? a.out + (size_t)b * 20 * TC : nullptr;  // null: the node-pool slot only
  bf16_t* o2 = a.x.pool ? reinterpret_cast<bf16_t*>(a.x.pool) + (size_t)b * a.x.pool_env_stride +
                              (size_t)a.x.pool_slot * 20 * TC
                        : nullptr;
  for (int u = 0; u < 640 / TPE; ++u) {
    const int i = u * TPE + t, p = i >> 5, c = i & 31;
    float f[8];
    unpack8<EL>(*reinterpret_cast<const uint4*>(lds + toff(t8::row8(e, p), c)), f);
    const uint4 r = make_uint4(pack_bf16x2((f[0] - mn) / den, (f[1] - mn) / den), pack_bf16x2((f[2] - mn) / den, (f[3] - mn) / den),
                               pack_bf16x2((f[4] - mn) / den, (f[5] - mn) / den), pack_bf16x2((f[6] - mn) / den, (f[7] - mn) / den));
    if (o1) *reinterpret_cast<uint4*>(o1 + p * TC + c * 8) = r;
    if (o2) *reinterpret_cast<uint4*>(o2 + p * TC + c * 8) = r;
  }
}

// one residual-tower conv (in place): k loop, barrier, write back, barrier
template <int EL, int NQ, bool RESID, class G = Geo45<NQ>>
__device__ __forceinline__ void tower8_conv(uint8_t* __restrict__ lds, const WNext& cur, const WNext& nxt, int ct0,
                                            const float* __restrict__ bconv, uint2 (&res)[T8<NQ>::NRT][t8::CT],
                                            uint4 (&bq)[t8::CT][t8d<NQ>], int lane, int ci) {
  f32x4 acc[T8<NQ>::NRT][t8::CT];
  tower8_acc<EL, NQ, RESID ? 1 : 0, false, t8::CT, G>(lds, cur, nxt, ct0, bconv, nullptr, nullptr, 0, res, bq, acc, lane, ci);
  __syncthreads();  // every wave has read the whole image
  TSTAMP(6 + 6 * ci);
  tower8_writeback<EL, NQ, !RESID>(lds, acc, res, 0, ct0, lane);
  __syncthreads();
  TSTAMP(7 + 6 * ci);
}

// tower convs' biases staged in LDS (dynamic shared memory after the image): 2 nblocks x 256 f32
constexpr int T8_MAX_BLOCKS = 24;

template <int EL, int NQ>
__global__ __launch_bounds__(t8::NT, 1) void tower8_kernel(TowerArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[T8<NQ>::BYTES];
  __shared__ long long envoff[T8<NQ>::E];
  __shared__ int acts[T8<NQ>::E];
  __shared__ float part[4 * 8 * 16];  // head partial sums [wave][env][output]
  __shared__ float lg[2 * 8 * 16];    // head logits [head][env][output]
  __shared__ float dec[2][8][4];      // decoded head outputs [head][env][output]
  extern __shared__ __attribute__((aligned(16))) float biasl[];  // [2 nblocks][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int env0 = blockIdx.x * T8<NQ>::E;
  const int nenv = min(T8<NQ>::E, a.B - env0);
  const int rows = nenv * 20;
  const bool pro = a.x.w0 != nullptr;
  const int ctw = wave * t8::CT;
  const uint4* wf = reinterpret_cast<const uint4*>(a.wf);
  constexpr size_t WCONV = (size_t)16 * TNS * 64;
  // the weight ring's first k steps fly while the image is staged
  uint4 bq[t8::CT][t8d<NQ>];
  TSTAMP(0);
#ifdef TOWER_STAMPS
  tstamp(TST_N - 3, true);
#endif
  // prologue loads in one round trip: the env's node-pool slot and action first (the oldest loads,
  // so waiting for them leaves the rest in flight), then the weight ring's first k steps and every
  // tower bias (at most BPT float4 per thread) before any of them is used. A per-element bias loop
  // (load, LDS store) waited one round trip per iteration, 7 at 14 blocks, behind the ring loads.
  int slot_b = 0, act_b = 0;
  const int b_own = env0 + (tid < nenv ? tid : 0);
  if (tid < T8<NQ>::E) {
    if (a.slot) slot_b = a.slot[b_own];
    if (pro) act_b = a.x.act[b_own];
  }
  const WNext first = wnext(pro ? a.x.w0 : a.wf, TNS, ctw);
  tower8_preload<t8::CT, NQ>(bq, first, lane);
  // where each wave's ring goes after the last tower conv: the epilogue conv it runs
  WNext epi = first;
  if (a.x.epilogue == 1) epi = wnext(a.x.we1, 8, ctw);
  // (epilogue 2 reloads its own 2-tile ring: the last tower conv's continuation loads re-read `first`)
  constexpr int BPT = (T8_MAX_BLOCKS * 2 * TC / 4 + t8::NT - 1) / t8::NT;
  const int n4 = a.nblocks * 2 * TC / 4;
  // (indices past the table are clamped to its last element, loads and stores alike: a store under
  // a condition makes the compiler sink its load into the branch and wait for it there)
  float4 bv[BPT];
#pragma unroll
  for (int u = 0; u < BPT; ++u)
    bv[u] = reinterpret_cast<const float4*>(a.bias)[min(u * t8::NT + tid, n4 - 1)];
  if (tid < T8<NQ>::E) {
    envoff[tid] = (long long)b_own * a.in_env_stride + (long long)slot_b * a.in_slot_stride;
    acts[tid] = act_b;
  }
#pragma unroll
  for (int u = 0; u < BPT; ++u) reinterpret_cast<float4*>(biasl)[min(u * t8::NT + tid, n4 - 1)] = bv[u];
  __syncthreads();
  {  // stage X: ROWS x 32 chunks, 10 per thread per batch (NQ batches)
#pragma unroll
    for (int h = 0; h < NQ; ++h) {
      uint4 v[10];
#pragma unroll
      for (int u = 0; u < 10; ++u) {
        const int i = (h * 10 + u) * t8::NT + tid;
        const int r = i >> 5, c = i & 31;
        const bool ok = r < rows;
        const int rr = ok ? r : 0;
        v[u] = Elt<EL>::from_bf16(*reinterpret_cast<const uint4*>(a.in + envoff[rr / 20] + (long long)(rr % 20) * TC + c * 8));
        if (!ok) v[u] = make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 10; ++u) {
        const int i = (h * 10 + u) * t8::NT + tid;
        const int r = i >> 5;
        *reinterpret_cast<uint4*>(lds + toff(t8::row8(r / 20, r % 20), i & 31)) = v[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) *reinterpret_cast<uint4*>(lds + T8<NQ>::LZ + (u * t8::NT + tid) * 16) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  TSTAMP(1);
  uint2 res[T8<NQ>::NRT][t8::CT];
  if (pro) {  // dynamics ConvBlock (in place)
    f32x4 acc[T8<NQ>::NRT][t8::CT];
    tower8_acc<EL, NQ, 2, false>(lds, first, wnext(a.wf, TNS, ctw), ctw, a.x.b0, a.x.act_bias, acts, a.x.A, res, bq, acc, lane);
    __syncthreads();
    tower8_writeback<EL, NQ, false>(lds, acc, res, 0, ctw, lane);
    __syncthreads();
  }
  for (int blk = 0; blk < a.nblocks; ++blk) {
    const WNext c1 = wnext(wf + (2 * blk) * WCONV, TNS, ctw), c2 = wnext(wf + (2 * blk + 1) * WCONV, TNS, ctw);
    const WNext c3 = blk + 1 < a.nblocks ? wnext(wf + (2 * blk + 2) * WCONV, TNS, ctw) : epi;
    tower8_conv<EL, NQ, false>(lds, c1, c2, ctw, biasl + (2 * blk) * TC, res, bq, lane, 2 * blk);
    tower8_conv<EL, NQ, true>(lds, c2, c3, ctw, biasl + (2 * blk + 1) * TC, res, bq, lane, 2 * blk + 1);
  }
  if (a.x.epilogue == 1) {  // dynamics: reward ConvBlock1x1, the scaled latent from X, then Linear + decode
    f32x4 acc[T8<NQ>::NRT][t8::CT];
    tower8_acc<EL, NQ, 0, true>(lds, epi, epi, ctw, a.x.be1, nullptr, nullptr, 0, res, bq, acc, lane);
    __syncthreads();
    tower8_scale<EL, NQ>(a, lds, env0, nenv, tid);  // reads X before the reward conv output replaces it
    __syncthreads();
    tower8_writeback<EL, NQ, false>(lds, acc, res, 0, ctw, lane);
    __syncthreads();
    const int hc0[2] = {0, 0}, hC[2] = {TC, 0}, kind[2] = {1, 0};
    tower_heads<EL, T8<NQ>::E, 4, true>(a, lds, 0, 1, hc0, hC, kind, part, lg, dec, env0, nenv, tid);
    return;
  }
  if (a.x.epilogue == 2) {  // prediction: policy 3x3 256->128 -> [0,128), value 1x1 256->128 -> [128,256),
    // each wave 2 of the 8 column tiles of both (balanced: a 3x3 on two waves beside a 1x1 on the other
    // two left two SIMDs idle for most of a conv)
    const int ctp = wave * 2;
    f32x4 accp[T8<NQ>::NRT][2], accv[T8<NQ>::NRT][2];
    uint4 bq2[2][t8d<NQ>];
    const WNext wp3 = wnext(a.x.we3, TNS, ctp), wv1 = wnext(a.x.we1, 8, ctp);
    tower8_preload<2, NQ>(bq2, wp3, lane);
    tower8_acc<EL, NQ, 0, false, 2>(lds, wp3, wv1, ctp, a.x.be3, nullptr, nullptr, 0, res, bq2, accp, lane);
    tower8_acc<EL, NQ, 0, true, 2>(lds, wv1, wv1, ctp, a.x.be1, nullptr, nullptr, 0, res, bq2, accv, lane);
    __syncthreads();
    tower8_writeback<EL, NQ, false, 2>(lds, accp, res, 0, ctp, lane);
    tower8_writeback<EL, NQ, false, 2>(lds, accv, res, 128, ctp, lane);
    __syncthreads();
    // the ucb factor tables go to LDS for the tree walk (`part` is free after the heads): loaded
    // here, stored after the heads, so the walk's per-level table reads are LDS reads
    const int ntab = a.tree.S + 1;
    const bool tab_lds = a.tree_on && ntab <= t8::NT;
    float tsq = 0.f, tct = 0.f;
    if (tab_lds && tid < ntab) { tsq = a.tree.sqrt_tab[tid]; tct = a.tree.c_tab[tid]; }
    const int hc0[2] = {0, 128}, hC[2] = {128, 128}, kind[2] = {0, 1};
    tower_heads<EL, T8<NQ>::E, 4, true>(a, lds, 0, 2, hc0, hC, kind, part, lg, dec, env0, nenv, tid);
    if (a.tree_on) {  // this simulation's backup and the next selection (mcts.py:136-234), per env
      __syncthreads();
      if (tab_lds && tid < ntab) { part[tid] = tsq; part[ntab + tid] = tct; }
      __syncthreads();
      if (tid < nenv) {
        const int b = env0 + tid;
        tree_backup_env(a.tree, a.tree_sim, b, a.tree_r[b], dec[1][tid][0], &dec[0][tid][0], a.tree_gamma);
        if (a.tree_sim + 1 < a.tree.S)
          tree_select_env(a.tree, a.tree_sim + 1, b, tab_lds ? part : nullptr, tab_lds ? part + ntab : nullptr);
      }
    }
    return;
  }
#pragma unroll 4
  for (int u = 0; u < 10 * NQ; ++u) {
    const int i = u * t8::NT + tid;
    const int r = i >> 5, c = i & 31;
    if (r < rows)
      *reinterpret_cast<uint4*>(a.out + (long long)(env0 + r / 20) * 20 * TC + (r % 20) * TC + c * 8) =
          Elt<EL>::to_bf16(*reinterpret_cast<const uint4*>(lds + toff(t8::row8(r / 20, r % 20), c)));
  }
  TSTAMP_END();
}

// ---------------------------------------------------------------------------------------------
// Representation tail (networks.py:86-99 after the 16x20 blocks, :271-280, _scale_state :314-328) in
// ONE launch: AvgPool2d 16x20 -> 8x10 while staging, nblocks ResidualBlock(256) at 8x10 with the
// activations LDS-resident, AvgPool2d -> 4x5 and the per-env min-max scale in the epilogue; the root
// latent goes to `out` and to node-pool slot 0. A workgroup owns 2 envs = 160 rows x 256 channels
// (Geo810: a 16-row tile is one latent column x of 2 envs x 8 rows) and runs tower8_kernel's k loop,
// weight ring and in-place convs. Pooling follows avgpool2_kernel's op order ((a + b) + c) + d, / 4,
// bf16; the scale follows scale_state_kernel: the unfused launch sequence, fused.
struct RepTailArgs {
  const bf16_t* in;          // [B][320][256]: the activations after the last 16x20 block
  bf16_t* out;               // [B][20][256] scaled root latent
  bf16_t* pool;              // optional: env b's slot 0 at pool + b * pool_env_stride
  long long pool_env_stride;
  const bf16_t* wf;          // 2 nblocks convs in the tower packing, back to back (+ pad)
  const float* bias;         // [2 nblocks][256]
  int nblocks, B;
};

__global__ __launch_bounds__(t8::NT, 1) void rep_tail_kernel(RepTailArgs a) {
  using G = Geo810;
  __shared__ __attribute__((aligned(16))) uint8_t lds[G::LZ + 16 * TROWB];  // image | 16 zero rows
  __shared__ float mm[2][2][2];                                             // [env][wave of env][min, max]
  extern __shared__ __attribute__((aligned(16))) float biasl[];             // [2 nblocks][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int env0 = blockIdx.x * 2;
  const int nenv = min(2, a.B - env0);
  const int ctw = wave * t8::CT;
  const uint4* wf = reinterpret_cast<const uint4*>(a.wf);
  constexpr size_t WCONV = (size_t)16 * TNS * 64;
  uint4 bq[t8::CT][t8d<2>];
  tower8_preload<t8::CT, 2>(bq, wnext(a.wf, TNS, ctw), lane);  // flies while the input is pooled and staged
  {
    const int n4 = a.nblocks * 2 * TC / 4;
    for (int i = tid; i < n4; i += t8::NT) reinterpret_cast<float4*>(biasl)[i] = reinterpret_cast<const float4*>(a.bias)[i];
  }
  // stage: 2 envs x 80 pooled positions x 32 chunks, 4 per thread per batch (4 x 16-B loads each)
#pragma unroll 1
  for (int i0 = 0; i0 < 2 * 80 * 32; i0 += 4 * t8::NT) {
    uint4 v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * t8::NT + tid, e = i / 2560, r = i - e * 2560, pp = r >> 5, c = r & 31;
      const int yo = pp / 10, xo = pp - yo * 10;
      const int eb = env0 + (e < nenv ? e : 0);
      const bf16_t* src = a.in + (size_t)eb * 320 * TC + (size_t)(2 * yo * 20 + 2 * xo) * TC + c * 8;
      v[u][0] = *reinterpret_cast<const uint4*>(src);
      v[u][1] = *reinterpret_cast<const uint4*>(src + TC);
      v[u][2] = *reinterpret_cast<const uint4*>(src + 20 * TC);
      v[u][3] = *reinterpret_cast<const uint4*>(src + 21 * TC);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * t8::NT + tid, e = i / 2560, r = i - e * 2560, pp = r >> 5, c = r & 31;
      const int yo = pp / 10, xo = pp - yo * 10;
      float f0[8], f1[8], f2[8], f3[8];
      unpack8<0>(v[u][0], f0); unpack8<0>(v[u][1], f1); unpack8<0>(v[u][2], f2); unpack8<0>(v[u][3], f3);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (((f0[j] + f1[j]) + f2[j]) + f3[j]) / 4.0f;
      uint4 w = make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]),
                           pack_bf16x2(o[6], o[7]));
      if (e >= nenv) w = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(lds + toff(xo * 16 + yo * 2 + e, c)) = w;
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) *reinterpret_cast<uint4*>(lds + G::LZ + (u * t8::NT + tid) * 16) = make_uint4(0, 0, 0, 0);
  __syncthreads();
  uint2 res[T8<2>::NRT][t8::CT];
  for (int blk = 0; blk < a.nblocks; ++blk) {
    const WNext c1 = wnext(wf + (2 * blk) * WCONV, TNS, ctw), c2 = wnext(wf + (2 * blk + 1) * WCONV, TNS, ctw);
    const WNext c3 = blk + 1 < a.nblocks ? wnext(wf + (2 * blk + 2) * WCONV, TNS, ctw) : c1;  // last: harmless
    tower8_conv<0, 2, false, G>(lds, c1, c2, ctw, biasl + (2 * blk) * TC, res, bq, lane, 2 * blk);
    tower8_conv<0, 2, true, G>(lds, c2, c3, ctw, biasl + (2 * blk + 1) * TC, res, bq, lane, 2 * blk + 1);
  }
  // epilogue: AvgPool2d 8x10 -> 4x5 (bf16), per-env min / max, the scaled latent. 128 threads per env,
  // 5 of its 640 chunks each
  const int e = tid >> 7, t = tid & 127;
  uint4 pv[5];
  float mn = INFINITY, mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int i = u * 128 + t, pp = i >> 5, c = i & 31, y4 = pp / 5, x4 = pp - y4 * 5;
    const int r00 = (2 * x4) * 16 + (2 * y4) * 2 + e;  // (2y, 2x); +16: x + 1; +2: y + 1
    float f0[8], f1[8], f2[8], f3[8];
    unpack8<0>(*reinterpret_cast<const uint4*>(lds + toff(r00, c)), f0);
    unpack8<0>(*reinterpret_cast<const uint4*>(lds + toff(r00 + 16, c)), f1);
    unpack8<0>(*reinterpret_cast<const uint4*>(lds + toff(r00 + 2, c)), f2);
    unpack8<0>(*reinterpret_cast<const uint4*>(lds + toff(r00 + 18, c)), f3);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (((f0[j] + f1[j]) + f2[j]) + f3[j]) / 4.0f;
    pv[u] = make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]), pack_bf16x2(o[6], o[7]));
    float g[8];
    unpack8<0>(pv[u], g);  // min / max of the bf16 pooled values, as scale_state_kernel reads them
#pragma unroll
    for (int j = 0; j < 8; ++j) { mn = fminf(mn, g[j]); mx = fmaxf(mx, g[j]); }
  }
  for (int o = 32; o > 0; o >>= 1) { mn = fminf(mn, __shfl_xor(mn, o)); mx = fmaxf(mx, __shfl_xor(mx, o)); }
  if (lane == 0) { mm[e][(t >> 6)][0] = mn; mm[e][(t >> 6)][1] = mx; }
  __syncthreads();
  mn = fminf(mm[e][0][0], mm[e][1][0]);
  mx = fmaxf(mm[e][0][1], mm[e][1][1]);
  if (e >= nenv) return;
  const float den = (mx - mn) + 1e-8f;
  const int b = env0 + e;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int i = u * 128 + t;
    float g[8];
    unpack8<0>(pv[u], g);
    const uint4 r = make_uint4(pack_bf16x2((g[0] - mn) / den, (g[1] - mn) / den), pack_bf16x2((g[2] - mn) / den, (g[3] - mn) / den),
                               pack_bf16x2((g[4] - mn) / den, (g[5] - mn) / den), pack_bf16x2((g[6] - mn) / den, (g[7] - mn) / den));
    *reinterpret_cast<uint4*>(a.out + (size_t)b * 20 * TC + i * 8) = r;
    if (a.pool) *reinterpret_cast<uint4*>(a.pool + (size_t)b * a.pool_env_stride + i * 8) = r;
  }
}

static thread_local int g_tower_variant = 0;  // (per thread: an acting thread beside the learner) 0 auto, 1 four-env kernel, 2 eight-env kernel, 3 four-env 4-wave

static size_t t8_dyn_lds(int nblocks) { return (size_t)nblocks * 2 * TC * sizeof(float); }

static int tower_ncu() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  return ncu;
}

}  // namespace

extern "C" {

#ifdef TOWER_STAMPS
int mzba_tower_stamps_read(unsigned long long* host, int nrows) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mz_tower_stamps), sizeof(unsigned long long) * TST_N * nrows);
}
#endif

// 0: pick by batch (default), 1: force the 4-env kernel, 2: force the 8-env kernel, 3: the 4-env
// 4-wave kernel (the 8-env kernel's structure on one env quad)
int mzba_tower_set_variant(int v) {
  if (v < 0 || v > 4) return -1;
  g_tower_variant = v;
  return 0;
}

// kernel used for batch B: 2 eight-env (B >= 8 x CUs: it halves the per-env weight stream but needs
// that many envs to fill the chip), else 3 four-env 4-wave (the 8-env kernel's code on one env quad:
// each wave 4 column tiles x 5 row tiles). Kernel 1 (four-env 8-wave) stays selectable: it was the
// default below 8 x CUs until the 4-wave kernels got the cross-conv weight ring and front-loaded A
// reads (B = 1024 acting loop, same box: 20.2k env-steps/s on kernel 1, 20.9k on kernel 3,
// profiles/r02/plan3_1024/). All take agent.pack_tower_conv weights.
//
// Plan 4 (towerp.hip, round 3): 16 envs per workgroup, one MFMA tile per latent pixel — the padding
// taps the column tiles of plans 1-3 run on zero rows are not issued (130 of 180 tile-taps per env
// instead of 156), bit-identical outputs. It needs 16 envs per CU to fill the chip: from B >= 16 x CUs.
int mzba_tower_plan(int B) {
  if (B <= 0) return -1;
  if (g_tower_variant) return g_tower_variant;
  const int ncu = tower_ncu();
  return B >= 16 * ncu ? 4 : (B >= 8 * ncu ? 2 : 3);
}

// device workspace bytes mzba_tower needs for batch B (0 for both current kernels)
long long mzba_tower_ws_bytes(int B) { return B > 0 ? 0 : -1; }

// nblocks residual blocks (256 ch, 4x5) fused; wf16: per conv [16][72][64][8] bf16, k steps in the
// (dx, dy) tap order of agent.pack_tower_conv (+8 KB pad after the last conv),
// bias: per conv [256] f32 (BN folded). in: env b at in + b*in_env_stride (+ slot[b]*in_slot_stride);
// out: [B][20][256]. ws: mzba_tower_ws_bytes(B) bytes of device scratch (may be null when 0).
int mzba_tower(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride, void* out,
               const void* wf16, const float* bias, int nblocks, int B, void* ws, long long ws_bytes,
               hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nblocks >= 1 && in && out && wf16 && bias, -1);
  const int plan = mzba_tower_plan(B);
  MZ_CHECK_ARG(plan > 0, -2);
  MZ_CHECK_ARG(plan == 1 || nblocks <= T8_MAX_BLOCKS, -5);  // tower8: bias table in LDS
  TowerArgs a{(const bf16_t*)in, in_env_stride, slot, in_slot_stride, (bf16_t*)out, (const bf16_t*)wf16, bias,
              nblocks, B, mzba_tower_ext{}, TreeArgs{}, 0, 0, 0.f, nullptr};
  (void)ws;
  (void)ws_bytes;
  if (plan == 4) return mzba_towerp(in, in_env_stride, slot, in_slot_stride, out, wf16, bias, nblocks, B, stream);
  if (plan == 2) {
    hipLaunchKernelGGL((tower8_kernel<0, 2>), dim3((B + 7) / 8), dim3(t8::NT), t8_dyn_lds(nblocks), stream, a);
  } else if (plan == 3) {
    hipLaunchKernelGGL((tower8_kernel<0, 1>), dim3((B + 3) / 4), dim3(t8::NT), t8_dyn_lds(nblocks), stream, a);
  } else {
    hipLaunchKernelGGL(tower_kernel<0>, dim3((B + TE - 1) / TE), dim3(TNT), 0, stream, a);
  }
  MZ_LAUNCH_CHECK();
  return 0;
}

// Representation tail (see include/mzba.h): 16x20 activations -> scaled 4x5 root latent, one launch.
int mzba_rep_tail(const void* in, void* out, void* pool, long long pool_env_stride, const void* wf16,
                  const float* bias, int nblocks, int B, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nblocks >= 1 && nblocks <= T8_MAX_BLOCKS && in && out && wf16 && bias && in != out, -1);
  RepTailArgs a{(const bf16_t*)in, (bf16_t*)out, (bf16_t*)pool, pool_env_stride, (const bf16_t*)wf16, bias, nblocks, B};
  hipLaunchKernelGGL(rep_tail_kernel, dim3((B + 1) / 2), dim3(t8::NT), t8_dyn_lds(nblocks), stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

// Dynamics / prediction step as one launch of the planned tower kernel (see include/mzba.h).
int mzba_tower_fused(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                     void* out, const void* wf16, const float* bias, int nblocks, int B, const mzba_tower_ext* ext,
                     hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nblocks >= 1 && in && wf16 && bias && ext, -1);
  int plan = ext->plan ? ext->plan : mzba_tower_plan(B);
  MZ_CHECK_ARG(plan >= 1 && plan <= 4, -4);
  if (plan == 4)  // bf16, or the fp16 dynamics net of config 5 (same packing, fp16 elements)
    return mzba_towerp_fused(in, in_env_stride, slot, in_slot_stride, out, wf16, bias, nblocks, B, ext, stream);
  MZ_CHECK_ARG(plan == 1 || nblocks <= T8_MAX_BLOCKS, -5);  // tower8: bias table in LDS
  const mzba_tower_ext& x = *ext;
  MZ_CHECK_ARG(x.epilogue >= 0 && x.epilogue <= 2 && (x.elem == 0 || x.elem == 1), -2);
  MZ_CHECK_ARG(!x.w0 || (x.b0 && x.act_bias && x.act && x.A > 0), -3);
  MZ_CHECK_ARG(x.epilogue != 0 || out, -3);
  MZ_CHECK_ARG(x.epilogue != 1 || ((out || x.pool) && x.we1 && x.be1 && x.lw[0] && x.lb[0] && x.dec[0] && x.lO[0] > 1 &&
                                   x.lO[0] <= 16), -3);
  MZ_CHECK_ARG(x.epilogue != 2 || (x.we3 && x.be3 && x.we1 && x.be1 && x.lw[0] && x.lw[1] && x.lb[0] && x.lb[1] &&
                                   x.dec[0] && x.dec[1] && x.lO[0] >= 1 && x.lO[0] <= 16 && x.lO[1] > 1 &&
                                   x.lO[1] <= 16), -3);
  TowerArgs a{(const bf16_t*)in, in_env_stride, slot, in_slot_stride, (bf16_t*)out, (const bf16_t*)wf16, bias,
              nblocks, B, x, TreeArgs{}, 0, 0, 0.f, nullptr};
  if (x.tree) {
    const mzba_tree_step& t = *x.tree;
    MZ_CHECK_ARG(x.epilogue == 2 && t.B == B && t.sim >= 0 && t.sim < t.S && t.r && t.nodes, -3);
    a.tree = TreeArgs{(Node*)t.nodes, t.root_sum, t.calls, t.leaf_parent, t.leaf_action, t.depth, t.path,
                      t.sqrt_tab, t.c_tab, t.B, t.S, t.env_offset, t.search_id, t.seed, t.ctx};
    a.tree_on = 1;
    a.tree_sim = t.sim;
    a.tree_gamma = t.gamma;
    a.tree_r = t.r;
  }
  const dim3 g8((B + 7) / 8), g4((B + TE - 1) / TE);
  if (x.elem == 1) {
    if (plan == 2) hipLaunchKernelGGL((tower8_kernel<1, 2>), g8, dim3(t8::NT), t8_dyn_lds(nblocks), stream, a);
    else if (plan == 3) hipLaunchKernelGGL((tower8_kernel<1, 1>), g4, dim3(t8::NT), t8_dyn_lds(nblocks), stream, a);
    else hipLaunchKernelGGL(tower_kernel<1>, g4, dim3(TNT), 0, stream, a);
  } else {
    if (plan == 2) hipLaunchKernelGGL((tower8_kernel<0, 2>), g8, dim3(t8::NT), t8_dyn_lds(nblocks), stream, a);
    else if (plan == 3) hipLaunchKernelGGL((tower8_kernel<0, 1>), g4, dim3(t8::NT), t8_dyn_lds(nblocks), stream, a);
    else hipLaunchKernelGGL(tower_kernel<0>, g4, dim3(TNT), 0, stream, a);
  }
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
