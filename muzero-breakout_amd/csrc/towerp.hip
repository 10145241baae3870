// Pixel-tiled residual tower (gfx950, bf16 MFMA): 16 envs per workgroup, one 16-row MFMA tile per
// latent PIXEL.
//
// tower8_kernel's tile is one latent column of an env quad (4 envs x 4 rows): a dy = +-1 tap shifts
// rows inside the tile, so 4 of its 16 rows multiply zero padding. The taps that fall on the 4x5
// latent's border are 50 of 180 per env (the reference's Conv2d(padding=1) computes them on zeros):
// a column tile skips the dx ones whole (39 of 45 tile-taps) but runs the dy ones, so 86.7 % of the
// algorithmic MFMA work executes and 72.2 % of it is useful. Here a tile is ONE pixel (y, x) of 16
// envs: every tap (dy, dx) maps pixel tile (y, x) onto pixel tile (y + dy, x + dx) whole, and the
// 50 border tile-taps are simply not issued (130 of 180 run, every row useful).
//
// A workgroup (4 waves, one per SIMD, 512 registers each) owns 16 envs x 20 pixels = 320 rows x 256
// channels for the whole tower:
//   * the activation image fills the CU's LDS (320 x 512 B = 160 KiB; no zero rows: nothing reads
//     padding). LDS row of (pixel p, env e) = 16 p + e, 16-B chunks XOR-swizzled by e, so a B
//     fragment (16 rows of one pixel, 8 channels per lane) is conflict-free for every tap;
//   * each wave owns 64 output channels (4 column tiles) x all 20 pixel tiles: 80 accumulators
//     (320 AGPRs), weights = MFMA A operand, activations = B operand (v_mfma_f32_16x16x32_bf16);
//   * a k step is one (dy, 32-channel) pair (24 per conv); within it the input pixel rows y' are
//     walked one at a time: the 5 B fragments of row y' (read once from LDS) feed the 13 valid
//     (dx, x') taps of each column tile into output row y' - dy: 52 MFMAs per 5 reads;
//   * weights: the tower packing ([col tile][pack step 24 (dx+1) + 8 (dy+1) + c][lane][8], 1 KB per
//     fragment, agent.pack_tower_conv) through a two-k-step ring of 24 fragments in registers, each
//     slot reloaded right after its last MFMA of the step; the ring runs across conv boundaries;
//   * two 32-channel passes per conv (a wave's column tiles 0-1, then 2-3: 40 accumulators each);
//     pass 0's result waits packed (ReLU, bf16) in registers for the write-back;
//   * in place: k loops, barrier, write-back (ReLU, bf16), barrier. The block input that conv2
//     adds back (the residual) cannot stay in LDS (no room beside the image): conv1's write-back
//     lifts it out of the image at the wave's own output positions, in the accumulator layout, into
//     registers (80 VGPRs), where conv2's accumulator init adds it.
// The kernel fills one CU per workgroup: B = 4096 is exactly one round on 256 CUs. EL (elt.h): bf16, or fp16
// for the fp16 dynamics net of config 5 (fp16 image, weights and MFMAs; latents in and out of HBM stay bf16,
// converted on staging and in the epilogues, as tower8_kernel<1, NQ>, bit for bit).
#include "common.h"
#include "tree_dev.h"
#include "elt.h"  // Elt<EL>: bf16 (EL 0) / fp16 (EL 1, the fp16 dynamics net of config 5) images and weights

#ifndef TP_STAGE
#define TP_STAGE 2  // staging batches per wave (2: two envs' 20 loads in flight at a time; 1: all four)
#endif

namespace {

namespace tp {
constexpr int E = 16;                  // envs per workgroup
constexpr int P = 20;                  // latent pixels (4 x 5)
constexpr int ROWS = E * P;            // 320
constexpr int C = 256;
constexpr int ROWB = C * 2;            // 512 B per LDS row
constexpr int IMG = ROWS * ROWB;       // 163 840 B: all of the CU's LDS
constexpr int PIX = E * ROWB;          // 8 KB per pixel tile
constexpr int NT = 256;                // 4 waves
constexpr int CT = 4;                  // column tiles per wave (64 output channels)
constexpr int TNS = 72;                // pack k steps per column tile of a 3x3 conv
constexpr int CTB = TNS * 1024;        // bytes per column tile of a 3x3 pack
MZ_DEV int off(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 15)) << 4); }
// ReLU on two packed bf16 / fp16 (the sign bit is the int16 sign: a signed 16-bit max with 0 clears
// negatives and -0): relu(round(x)) == round(relu(x)) for round-to-nearest, so this is the f32 ReLU
// before the conversion, bit for bit
MZ_DEV uint32_t relu_pk(uint32_t u) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(u));
  return r;
}
}  // namespace tp

#ifdef TOWERP_STAMPS
// diagnostic build only (make towerp-stamps -> libmzba_pstamp.so, tools/stamp_towerp.py): s_memtime at
// the phase boundaries, per workgroup and wave. 0 entry, 1 after staging; conv ci (0-based, the
// dynamics prologue conv included): 2 + 5 ci + {0 start, 1 pass 0 k loop done, 2 pass 1 k loop done,
// 3 after the first barrier, 4 after the write-back barrier}; 160.. epilogue phases; PST_N - 3 / - 2
// s_memrealtime at entry / exit, PST_N - 1 s_memtime at exit
constexpr int PST_N = 192, PST_WG = 256;
__device__ unsigned long long mz_towerp_stamps[PST_WG * 4][PST_N];
MZ_DEV void pstamp(int k, bool real = false) {
  if ((threadIdx.x & 63) == 0 && blockIdx.x < PST_WG && k < PST_N)
    mz_towerp_stamps[blockIdx.x * 4 + (threadIdx.x >> 6)][k] = real ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
}
#define PSTAMP(k) pstamp(k)
#else
#define PSTAMP(k) \
  do {            \
  } while (0)
#endif

// A wave's view of a 3x3 weight pack: buffer resource at the wave's first column tile; a fragment
// load takes the lane's offset in one VGPR and the (column tile, pack step) offset in an SGPR
struct TPW {
  __amdgpu_buffer_rsrc_t rs;
  MZ_DEV uint4 ld(int ct, int step, int lane) const {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, ct * tp::CTB + step * 1024, 0));
  }
};
MZ_DEV TPW tpw(const void* pack, int ct0) {
  const uint4* p = reinterpret_cast<const uint4*>(pack) + (size_t)ct0 * tp::TNS * 64;
  return TPW{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(p), 0, 0x7fffffff, 0x00020000)};
}

MZ_DEV TPW tpw1(const void* pack, int ct0) {  // a 1x1 pack (8 k steps per column tile)
  const uint4* p = reinterpret_cast<const uint4*>(pack) + (size_t)ct0 * 8 * 64;
  return TPW{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(p), 0, 0x7fffffff, 0x00020000)};
}

// Ring of one wave: bq[k step parity][dx + 1][column tile of the pass]; k step s of a pass uses
// pack steps 24 (dx + 1) + s, slot parity s & 1. The kernel's first two steps are preloaded; every
// later step is loaded by the step two before it — across pass and conv boundaries, the next pass's
// steps 0 and 1 (`nxt`: the other column-tile pair of the same conv, or the next conv's first pair).
MZ_DEV void tp_preload(uint4 (&bq)[2][3][2], const TPW& w, int lane) {
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) bq[cc][d][ct] = w.ld(ct, 24 * d + cc, lane);
}

// The 8 k steps (channel steps c = 0..7) of latent row shift dy = DYI - 1 for one pass (2 column
// tiles). Input pixel rows y' = YLO..YHI (those that are y + dy of an output row y); fragments of
// row y' at lds + lb + xo(c) + (5 y' + x') PIX with xo(c) = ((4c + q) ^ n) << 4 (lane row n, k
// quarter q). fa holds the first row step's fragments on entry and the next dy's first on exit
// (after dy = +1: the pass's own first ones again, i.e. the next pass's if the image is unchanged).
template <int EL, int DYI>
__device__ __forceinline__ void tp_dy(const uint8_t* __restrict__ lds, int lb, int q, int n, const TPW& cur,
                                      const TPW& nxt, uint4 (&bq)[2][3][2], f32x4 (&acc)[tp::P][2],
                                      typename Elt<EL>::v8 (&fa)[5], typename Elt<EL>::v8 (&fb)[5], int lane) {
  typedef typename Elt<EL>::v8 V8;
  constexpr int DY = DYI - 1;
  constexpr int YLO = DY < 0 ? 0 : DY, YHI = DY > 0 ? 3 : 3 + DY, NY = YHI - YLO + 1;
  constexpr int NYLO = DYI == 0 ? 0 : (DYI == 1 ? 1 : 0);  // first input row of the next dy loop
#pragma unroll 1
  for (int cp = 0; cp < 4; ++cp) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int c = 2 * cp + cc, s = 8 * DYI + c;
      const bool wrap = cc == 1 && cp == 3;  // the next k step opens the next dy loop
      const int cn = wrap ? 0 : c + 1;
      const int xc = lb + (((4 * c + q) ^ n) << 4), xn = lb + (((4 * cn + q) ^ n) << 4);
      const int ynext = wrap ? NYLO : YLO;
      // ring slots of this step reload pack step 24 d + s + 2 (past 23: the next pass's 24 d + s - 22)
      int st = s + 2;
      __amdgpu_buffer_rsrc_t rs = cur.rs;
      if (DYI == 2) {
        rs = st >= 24 ? nxt.rs : cur.rs;
        st = st >= 24 ? st - 24 : st;
      }
#pragma unroll
      for (int yi = 0; yi < NY; ++yi) {
        const int yp = YLO + yi;
        const int nb = yi + 1 < NY ? xc + 5 * (yp + 1) * tp::PIX : xn + 5 * ynext * tp::PIX;
        const bool last = yi == NY - 1;
        auto row = [&](const V8(&f)[5], V8(&fn)[5]) {
          V8 w[3][2];
#pragma unroll
          for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) w[d][ct] = __builtin_bit_cast(V8, bq[cc][d][ct]);
#pragma unroll
          for (int xp = 0; xp < 5; ++xp)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
              acc[(yp - DY) * 5 + xp][ct] = Elt<EL>::mfma(w[1][ct], f[xp], acc[(yp - DY) * 5 + xp][ct]);
#pragma unroll
          for (int xp = 0; xp < 5; ++xp) fn[xp] = *reinterpret_cast<const V8*>(lds + nb + xp * tp::PIX);
#pragma unroll
          for (int xp = 0; xp < 4; ++xp)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
              acc[(yp - DY) * 5 + xp + 1][ct] = Elt<EL>::mfma(w[0][ct], f[xp], acc[(yp - DY) * 5 + xp + 1][ct]);
#pragma unroll
          for (int xp = 1; xp < 5; ++xp)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
              acc[(yp - DY) * 5 + xp - 1][ct] = Elt<EL>::mfma(w[2][ct], f[xp], acc[(yp - DY) * 5 + xp - 1][ct]);
          if (last) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
              for (int d = 0; d < 3; ++d)
                bq[cc][d][ct] = __builtin_bit_cast(
                    uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, ct * tp::CTB + (24 * d + st) * 1024, 0));
          }
          // after 8 of the 10 dx = 0 MFMAs, the next row's 5 reads ride in the next 5 MFMA slots
          __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 13, 0);
          if (last) __builtin_amdgcn_sched_group_barrier(0x020, 6, 0);
          __builtin_amdgcn_sched_barrier(0);
        };
        if (((cc * NY + yi) & 1) == 0)
          row(fa, fb);
        else
          row(fb, fa);
      }
    }
  }
}

struct TPArgs {
  const bf16_t* in;
  long long in_env_stride;
  const int32_t* slot;
  long long in_slot_stride;
  bf16_t* out;        // [B][20][256]
  const bf16_t* wf;   // per conv [16 col tiles][72][64][8], convs back to back (+ 8 KB pad)
  const float* bias;  // per conv [256]
  int nblocks;
  int B;
  mzba_tower_ext x;   // fused prologue / epilogue (tower.hip's TowerArgs semantics)
  TreeArgs tree;      // prediction epilogue: backup(tree_sim) + select(tree_sim + 1) per env
  int tree_on, tree_sim;
  float tree_gamma;
  const float* tree_r;
};

// Accumulator init of one pixel of a pass; its channels are chb + 16 ct + 4q + i of the lane's row
// (pixel p, env n). MODE 0: bias; 1: bias + res (bf16 residual in registers); 2: bias + the dynamics
// action bias table act_bias[pixel][act][256] (the one-hot action planes folded, tower.hip MODE 2).
template <int EL, int MODE>
MZ_DEV void tp_init1(f32x4 (&acc)[2], const float4 (&bias)[2], int chb, const uint2 (&res)[2],
                     const float* __restrict__ actb, int act, int A, int q, int p) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int ch = chb + 16 * ct + 4 * q;
    const float4 b4 = bias[ct];
    f32x4 v = {b4.x, b4.y, b4.z, b4.w};
    if (MODE == 1) {
      const uint2 r = res[ct];
      v[0] += Elt<EL>::lo(r.x); v[1] += Elt<EL>::hi(r.x);
      v[2] += Elt<EL>::lo(r.y); v[3] += Elt<EL>::hi(r.y);
    } else if (MODE == 2) {
      const float4 t = *reinterpret_cast<const float4*>(actb + ((size_t)p * A + act) * tp::C + ch);
      v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
    }
    acc[ct] = v;
  }
}
template <int EL, int MODE>
MZ_DEV void tp_init(f32x4 (&acc)[tp::P][2], const float4 (&bias)[2], int chb, const uint2 (&res)[tp::P][2],
                    const float* __restrict__ actb, int act, int A, int q) {
#pragma unroll
  for (int p = 0; p < tp::P; ++p) tp_init1<EL, MODE>(acc[p], bias, chb, res[p], actb, act, A, q, p);
}
// the initialised accumulators pinned to AGPRs before a k loop (left to the allocator the loop-carried
// accumulators move between the register files on every iteration)
MZ_DEV void tp_pin(f32x4 (&acc)[tp::P][2]) {
#pragma unroll
  for (int p = 0; p < tp::P; ++p)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) asm volatile("" : "+a"(acc[p][ct]));
}

// the lane's bias values of a pass whose first channel is chb
MZ_DEV void tp_bias(float4 (&b)[2], const float* __restrict__ bias, int chb, int q) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) b[ct] = *reinterpret_cast<const float4*>(bias + chb + 16 * ct + 4 * q);
}

// k loop of a 3x3 pass (weights in the ring, fa = its first fragments)
template <int EL>
MZ_DEV void tp_k3(const uint8_t* __restrict__ lds, int lb, int q, int n, const TPW& cur, const TPW& nxt,
                  uint4 (&bq)[2][3][2], typename Elt<EL>::v8 (&fa)[5], typename Elt<EL>::v8 (&fb)[5],
                  f32x4 (&acc)[tp::P][2], int lane) {
  tp_dy<EL, 0>(lds, lb, q, n, cur, nxt, bq, acc, fa, fb, lane);
  tp_dy<EL, 1>(lds, lb, q, n, cur, nxt, bq, acc, fa, fb, lane);
  tp_dy<EL, 2>(lds, lb, q, n, cur, nxt, bq, acc, fa, fb, lane);
}

// k loop of a 1x1 pass (centre tap: every pixel tile, 8 channel steps); the pack has 8 k steps per
// column tile, the pass's two tiles at w (loaded here: an epilogue conv, once per launch)
template <int EL>
MZ_DEV void tp_k1(const uint8_t* __restrict__ lds, int lb, int q, int n, const TPW& w, f32x4 (&acc)[tp::P][2],
                  int lane) {
  typedef typename Elt<EL>::v8 V8;
  uint4 wq[8][2];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      wq[c][ct] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w.rs, lane * 16, ct * 8192 + c * 1024, 0));
  // 32 steps (channel step c, pixel row yp), each 5 B fragments -> 10 MFMAs; the next step's fragments
  // are read during the current step's MFMAs (double-buffered: a read per step waited on its own LDS
  // round trip, 20 k cycles for the reward conv's two passes against a 10 k MFMA floor). Per accumulator
  // the channel steps stay in ascending order.
  V8 fa[5], fb[5];
  auto rd = [&](int k, V8(&f)[5]) {
    const int xc = lb + (((4 * (k >> 2) + q) ^ n) << 4), yp = k & 3;
#pragma unroll
    for (int xp = 0; xp < 5; ++xp) f[xp] = *reinterpret_cast<const V8*>(lds + xc + (5 * yp + xp) * tp::PIX);
  };
  rd(0, fa);
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    auto step = [&](const V8(&f)[5], V8(&fn)[5]) {
      const int c = k >> 2, yp = k & 3;
      if (k + 1 < 32) rd(k + 1, fn);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int xp = 0; xp < 5; ++xp)
          acc[5 * yp + xp][ct] = Elt<EL>::mfma(__builtin_bit_cast(V8, wq[c][ct]), f[xp], acc[5 * yp + xp][ct]);
      if (k + 1 < 32) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 5, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    if (k & 1)
      step(fb, fa);
    else
      step(fa, fb);
  }
}

template <int EL>
MZ_DEV uint2 tp_pack(const f32x4& a) {
  return make_uint2(tp::relu_pk(Elt<EL>::pack2(a[0], a[1])), tp::relu_pk(Elt<EL>::pack2(a[2], a[3])));
}
// byte offset (in the image) of the lane's 4 channels ch..ch+3 of pixel 0, row n
MZ_DEV int tp_cofs(int ch, int n) { return n * tp::ROWB + (((ch >> 3) ^ n) << 4) + ((ch & 7) << 1); }

template <int EL>
MZ_DEV void tp_first_frags(const uint8_t* __restrict__ lds, int lb, int q, int n, typename Elt<EL>::v8 (&fa)[5]) {
  const int x0 = lb + ((q ^ n) << 4);  // dy = -1: first input row y' = 0, channel step 0
#pragma unroll
  for (int xp = 0; xp < 5; ++xp) fa[xp] = *reinterpret_cast<const typename Elt<EL>::v8*>(lds + x0 + xp * tp::PIX);
}

// One 3x3 256 -> 256 conv, in place: two passes (the wave's column tiles 0-1, then 2-3), barrier,
// write-back (ReLU, bf16), barrier. MODE as tp_init; SAVE (conv1 of a block): the write-back first
// lifts the block input at the wave's output positions into res (conv2's residual).
// w: this conv's pack; wn: where the ring goes after it (the next conv's first pass). bc holds this
// conv's pass-0 bias on entry and the next conv's (nbias) on exit; every bias is loaded one pass
// ahead, so no pass starts with a global round trip.
template <int EL, int MODE, bool SAVE>
__device__ __forceinline__ void tp_conv(uint8_t* __restrict__ lds, const uint4* w, const TPW& wn,
                                        const float* __restrict__ bias, float4 (&bc)[2], const float* __restrict__ nbias,
                                        uint2 (&res)[2][tp::P][2],
                                        const float* __restrict__ actb, int act, int A, uint4 (&bq)[2][3][2], int lane,
                                        int wave, int ci) {
  const int q = lane >> 4, n = lane & 15;
  const int lb = n * tp::ROWB;
  const int ct0 = tp::CT * wave;
  const TPW w0 = tpw(w, ct0), w1 = tpw(w, ct0 + 2);
  PSTAMP(2 + 5 * ci);
  typename Elt<EL>::v8 fa[5], fb[5];
  tp_first_frags<EL>(lds, lb, q, n, fa);
  uint2 out0[tp::P][2];
  f32x4 acc[tp::P][2];
  tp_init<EL, MODE>(acc, bc, 64 * wave, res[0], actb, act, A, q);
  tp_pin(acc);
  float4 b1[2];  // pass 1's bias, loaded ahead of pass 0's k loop
  tp_bias(b1, bias, 64 * wave + 32, q);
  tp_k3<EL>(lds, lb, q, n, w0, w1, bq, fa, fb, acc, lane);
  PSTAMP(3 + 5 * ci);
  // pass 0's accumulators out (ReLU, bf16, held in registers until the write-back) and pass 1's in,
  // pixel by pixel: each pixel's residual registers are freed as its packed output appears, so the
  // live register count stays flat through the transition (packing all, then initialising all,
  // spilled part of the packed output)
#pragma unroll
  for (int p = 0; p < tp::P; ++p) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) out0[p][ct] = tp_pack<EL>(acc[p][ct]);
    tp_init1<EL, MODE>(acc[p], b1, 64 * wave + 32, res[1][p], actb, act, A, q, p);
    __builtin_amdgcn_sched_barrier(0);
  }
  tp_pin(acc);
  tp_bias(bc, nbias, 64 * wave, q);  // the next conv's pass-0 bias, ahead of pass 1's k loop
  tp_k3<EL>(lds, lb, q, n, w1, wn, bq, fa, fb, acc, lane);
  PSTAMP(4 + 5 * ci);
  __syncthreads();  // every wave has read the whole image
  PSTAMP(5 + 5 * ci);
  int cofs[tp::CT];
#pragma unroll
  for (int ct = 0; ct < tp::CT; ++ct) cofs[ct] = tp_cofs(64 * wave + 16 * ct + 4 * q, n);
  // one pixel at a time (a scheduling barrier per pixel: hoisting every accumulator read ahead of the
  // stores spilled the packed first-pass output)
#pragma unroll
  for (int p = 0; p < tp::P; ++p) {
#pragma unroll
    for (int ct = 0; ct < tp::CT; ++ct) {
      uint2* ptr = reinterpret_cast<uint2*>(lds + p * tp::PIX + cofs[ct]);
      if (SAVE) res[ct >> 1][p][ct & 1] = *ptr;
      *ptr = ct < 2 ? out0[p][ct] : tp_pack<EL>(acc[p][ct - 2]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  PSTAMP(6 + 5 * ci);
}

// Linear heads over the image (networks.py:147, 207, 221): head h reads image channels
// [hc0[h], hc0[h] + hC[h]) of the 20 pixels of each env, K = 20 hC[h] in (pixel, channel) order against
// bf16 weights lw[h][16][K]; one v_mfma_f32_16x16x32_bf16 per 32-deep k step (A rows = the 16 envs,
// B cols = outputs), k steps split over the 4 waves. The image is dead after the MFMAs: the partial
// sums, logits and decoded outputs go to LDS over it (scratch floats: part [2][4][16][16], lg
// [2][16][16], dec [2][16][4]). Then softmax (kind 0) or support decode (1), as tower_heads.
constexpr int TPH_PART = 0, TPH_LG = 2048, TPH_DEC = 2560, TPH_TAB = 2688;  // float offsets in the scratch
// NH heads over channel widths C0 / C1: every weight fragment of the wave (its k steps wave + 4u of
// each head, 40 in all) is loaded in one batch before the first MFMA — one L2 round trip instead of
// one per 10-step batch; the MFMAs run in tower_heads' order (k steps ascending per head)
template <int EL, int NH, int C0, int C1>
MZ_DEV void tp_heads(const TPArgs& a, uint8_t* __restrict__ lds, const int (&hc0)[2], const int (&kind)[2], int env0,
                     int nenv, int tid) {
  constexpr int NU0 = 20 * C0 / 32 / 4, NU1 = NH > 1 ? 20 * C1 / 32 / 4 : 0, NU = NU0 + NU1;
  static_assert(NU <= 40, "head weight batch");
  const int nh = NH;
  const int lane = tid & 63, wave = tid >> 6, q = lane >> 4, el = lane & 15;
  typedef typename Elt<EL>::v8 V8;
  f32x4 hacc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  V8 bv[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int hd = u < NU0 ? 0 : 1, K = 20 * (hd ? C1 : C0), s = wave + 4 * (hd ? u - NU0 : u);
    bv[u] = *reinterpret_cast<const V8*>(reinterpret_cast<const bf16_t*>(a.x.lw[hd]) + (size_t)el * K + s * 32 + q * 8);
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int hd = u < NU0 ? 0 : 1, C = hd ? C1 : C0, s = wave + 4 * (hd ? u - NU0 : u);
    const int k = s * 32 + q * 8;
    const int pos = k / C, c = hc0[hd] + (k - pos * C);
    const V8 av = *reinterpret_cast<const V8*>(lds + tp::off(pos * tp::E + el, c >> 3));
    hacc[hd] = Elt<EL>::mfma(av, bv[u], hacc[hd]);
  }
  __syncthreads();  // the image is dead: LDS becomes head scratch
  float* sc = reinterpret_cast<float*>(lds);
  float* part = sc + TPH_PART;
  float* lg = sc + TPH_LG;
  float* dec = sc + TPH_DEC;
#pragma unroll
  for (int hd = 0; hd < 2; ++hd)
    if (hd < nh)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[((hd * 4 + wave) * 16 + 4 * q + i) * 16 + el] = hacc[hd][i];  // D[env 4q + i][out el]
  __syncthreads();
  for (int hd = 0; hd < nh; ++hd) {
    const int e = tid >> 4, o = tid & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v = v + part[((hd * 4 + w) * 16 + e) * 16 + o];
    if (o < a.x.lO[hd]) lg[(hd * 16 + e) * 16 + o] = v + a.x.lb[hd][o];
  }
  __syncthreads();
  if (tid < 16 * nh) {
    const int hd = tid >> 4, e = tid & 15, b = env0 + e;
    if (e < nenv) {
      const int O = a.x.lO[hd];
      float l[16];
      for (int o = 0; o < O; ++o) {
        l[o] = lg[(hd * 16 + e) * 16 + o];
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
          if (o < 4) dec[(hd * 16 + e) * 4 + o] = p;
        }
      } else {
        const float d = decode_support(l, O, a.x.smin, a.x.smax);
        a.x.dec[hd][b] = d;
        dec[(hd * 16 + e) * 4] = d;
      }
    }
  }
}

// _scale_state (networks.py:314-328) of the image: per env (h - min) / (max - min + 1e-8) in f32,
// bf16 to out (and the node-pool slot); 16 threads per env, 40 chunks each
template <int EL>
MZ_DEV void tp_scale(const TPArgs& a, const uint8_t* __restrict__ lds, int env0, int nenv, int tid) {
  const int e = tid >> 4, t = tid & 15;
  // min / max on the packed 16-bit words: X is a ReLU output (relu_pk: +0 for every non-positive), and
  // non-negative bf16 / fp16 values order as their unsigned bit patterns, so v_pk_min_u16 /
  // v_pk_max_u16 over two values at a time give the f32 min / max of the unpacked values exactly
  uint32_t mn2 = 0xffffffffu, mx2 = 0u;
#pragma unroll 8
  for (int u = 0; u < 40; ++u) {
    const int i = u * 16 + t, p = i >> 5, c = i & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(lds + tp::off(p * tp::E + e, c));
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      asm("v_pk_min_u16 %0, %1, %2" : "=v"(mn2) : "v"(mn2), "v"(w4[j]));
      asm("v_pk_max_u16 %0, %1, %2" : "=v"(mx2) : "v"(mx2), "v"(w4[j]));
    }
  }
  const uint32_t mnh = min(mn2 & 0xffffu, mn2 >> 16), mxh = max(mx2 & 0xffffu, mx2 >> 16);
  float mn = Elt<EL>::lo(mnh), mx = Elt<EL>::lo(mxh);
  for (int o = 8; o > 0; o >>= 1) { mn = fminf(mn, __shfl_xor(mn, o)); mx = fmaxf(mx, __shfl_xor(mx, o)); }
  if (e >= nenv) return;
  const float den = (mx - mn) + 1e-8f;
  // x / den correctly rounded as f32((double)x * R), R = f64(1 / den): the product is within 2^-52
  // (relative) of the exact quotient, while a quotient of two f32 lies at least 2^-49 from any f32
  // rounding midpoint (a = mu den would need a 25-bit odd significand times a 24-bit one to fit in
  // 24 bits), so the rounding is the IEEE division's, bit for bit, at 3 instructions per element
  // instead of the ~10 of the f32 division sequence
  const double rden = 1.0 / (double)den;
  auto dv = [&](float x) { return (float)((double)(x - mn) * rden); };
  const int b = env0 + e;
  bf16_t* o1 = a.out ? a.out + (size_t)b * 20 * tp::C : nullptr;  // null: the node-pool slot only
  bf16_t* o2 = a.x.pool ? reinterpret_cast<bf16_t*>(a.x.pool) + (size_t)b * a.x.pool_env_stride +
                              (size_t)a.x.pool_slot * 20 * tp::C
                        : nullptr;
#pragma unroll 4
  for (int u = 0; u < 40; ++u) {
    const int i = u * 16 + t, p = i >> 5, c = i & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(lds + tp::off(p * tp::E + e, c));
    float f[8];
    unpack8<EL>(v, f);
    const uint4 r = make_uint4(pack_bf16x2(dv(f[0]), dv(f[1])), pack_bf16x2(dv(f[2]), dv(f[3])),
                               pack_bf16x2(dv(f[4]), dv(f[5])), pack_bf16x2(dv(f[6]), dv(f[7])));
    if (o1) *reinterpret_cast<uint4*>(o1 + p * tp::C + c * 8) = r;
    if (o2) *reinterpret_cast<uint4*>(o2 + p * tp::C + c * 8) = r;
  }
}

template <int EL>
__global__ __launch_bounds__(tp::NT, 1) void towerp_kernel(TPArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[tp::IMG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, n = lane & 15, lb = n * tp::ROWB;
  const int env0 = blockIdx.x * tp::E;
  const int nenv = min(tp::E, a.B - env0);
  const uint4* wf = reinterpret_cast<const uint4*>(a.wf);
  constexpr size_t WCONV = (size_t)16 * tp::TNS * 64;  // uint4 per conv pack
  const bool pro = a.x.w0 != nullptr;
  const int ct0 = tp::CT * wave;
  PSTAMP(0);
#ifdef TOWERP_STAMPS
  pstamp(PST_N - 3, true);
#endif
  uint4 bq[2][3][2];
  tp_preload(bq, tpw(pro ? a.x.w0 : a.wf, ct0), lane);
  // the lane's env (row n of every pixel tile): its action for the dynamics ConvBlock's bias table
  const int act = pro ? a.x.act[env0 + (n < nenv ? n : 0)] : 0;
  // stage: wave w owns envs 4w .. 4w + 3, one env (640 contiguous 16-B chunks) per batch of 10 loads;
  // TP_STAGE batches of 4 / TP_STAGE envs in flight at once
  constexpr int SB = 4 / TP_STAGE;
#pragma unroll
  for (int h = 0; h < TP_STAGE; ++h) {
    uint4 v[10 * SB];
#pragma unroll
    for (int bb = 0; bb < SB; ++bb) {
      const int e = 4 * wave + SB * h + bb;
      const bool ok = e < nenv;
      const int b = env0 + (ok ? e : 0);
      const long long eo = (long long)b * a.in_env_stride + (a.slot ? (long long)a.slot[b] * a.in_slot_stride : 0);
#pragma unroll
      for (int u = 0; u < 10; ++u) {
        v[bb * 10 + u] = Elt<EL>::from_bf16(*reinterpret_cast<const uint4*>(a.in + eo + (long long)(u * 64 + lane) * 8));
        if (!ok) v[bb * 10 + u] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int bb = 0; bb < SB; ++bb) {
      const int e = 4 * wave + SB * h + bb;
#pragma unroll
      for (int u = 0; u < 10; ++u) {
        const int cj = u * 64 + lane;
        *reinterpret_cast<uint4*>(lds + tp::off((cj >> 5) * tp::E + e, cj & 31)) = v[bb * 10 + u];
      }
    }
  }
  __syncthreads();
  PSTAMP(1);
  uint2 res[2][tp::P][2];
  const int nconv = 2 * a.nblocks;
  // where the ring goes after the last tower conv: the prediction epilogue's policy conv, else
  // anything in bounds (the first tower conv)
  const TPW after = a.x.epilogue == 2 ? tpw(a.x.we3, 2 * wave) : tpw(wf, ct0);
  float4 bc[2];
  tp_bias(bc, pro ? a.x.b0 : a.bias, 64 * wave, q);
  if (pro)  // dynamics ConvBlock 259 -> 256 (in place)
    tp_conv<EL, 2, false>(lds, reinterpret_cast<const uint4*>(a.x.w0), tpw(wf, ct0), a.x.b0, bc, a.bias, res, a.x.act_bias,
                      act, a.x.A, bq, lane, wave, 0);
  const int ci0 = pro ? 1 : 0;
  for (int blk = 0; blk < a.nblocks; ++blk) {
    const int k1 = 2 * blk, k2 = k1 + 1;
    const TPW w3 = k2 + 1 < nconv ? tpw(wf + (k2 + 1) * WCONV, ct0) : after;
    tp_conv<EL, 0, true>(lds, wf + k1 * WCONV, tpw(wf + k2 * WCONV, ct0), a.bias + k1 * tp::C, bc, a.bias + k2 * tp::C, res,
                     nullptr, 0, 0, bq, lane, wave, ci0 + k1);
    tp_conv<EL, 1, false>(lds, wf + k2 * WCONV, w3, a.bias + k2 * tp::C, bc, a.bias + (k2 + 1 < nconv ? k2 + 1 : k2) * tp::C,
                      res, nullptr, 0, 0, bq, lane, wave, ci0 + k2);
  }
  if (a.x.epilogue == 1) {  // dynamics: reward ConvBlock1x1, the scaled latent from X, then Linear + decode
    uint2 out0[tp::P][2];
    {
      f32x4 acc[tp::P][2];
      float4 b4[2];
      tp_bias(b4, a.x.be1, 64 * wave, q);
      tp_init<EL, 0>(acc, b4, 64 * wave, res[0], nullptr, 0, 0, q);
      tp_pin(acc);
      tp_k1<EL>(lds, lb, q, n, tpw1(a.x.we1, ct0), acc, lane);
#pragma unroll
      for (int p = 0; p < tp::P; ++p)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) out0[p][ct] = tp_pack<EL>(acc[p][ct]);
    }
    f32x4 acc[tp::P][2];
    float4 b4[2];
    tp_bias(b4, a.x.be1, 64 * wave + 32, q);
    tp_init<EL, 0>(acc, b4, 64 * wave + 32, res[0], nullptr, 0, 0, q);
    tp_pin(acc);
    tp_k1<EL>(lds, lb, q, n, tpw1(a.x.we1, ct0 + 2), acc, lane);
    PSTAMP(160);
    __syncthreads();
    tp_scale<EL>(a, lds, env0, nenv, tid);  // reads X before the reward conv output replaces it
    __syncthreads();
    PSTAMP(161);
#pragma unroll
    for (int p = 0; p < tp::P; ++p)
#pragma unroll
      for (int ct = 0; ct < tp::CT; ++ct)
        *reinterpret_cast<uint2*>(lds + p * tp::PIX + tp_cofs(64 * wave + 16 * ct + 4 * q, n)) =
            ct < 2 ? out0[p][ct] : tp_pack<EL>(acc[p][ct - 2]);
    __syncthreads();
    const int hc0[2] = {0, 0}, kind[2] = {1, 0};
    PSTAMP(162);
    tp_heads<EL, 1, tp::C, 0>(a, lds, hc0, kind, env0, nenv, tid);
    PSTAMP(163);
#ifdef TOWERP_STAMPS
    pstamp(PST_N - 2, true);
    pstamp(PST_N - 1);
#endif
    return;
  }
  if (a.x.epilogue == 2) {  // prediction: policy 3x3 256->128 -> [0,128), value 1x1 256->128 -> [128,256):
    // each wave its 2 of the 8 column tiles of both (pack column tiles 2w, 2w + 1)
    uint2 pol[tp::P][2];
    {
      f32x4 acc[tp::P][2];
      typename Elt<EL>::v8 fa[5], fb[5];
      tp_first_frags<EL>(lds, lb, q, n, fa);
      float4 b4[2];
      tp_bias(b4, a.x.be3, 32 * wave, q);
      tp_init<EL, 0>(acc, b4, 32 * wave, res[0], nullptr, 0, 0, q);
      tp_pin(acc);
      const TPW wp = tpw(a.x.we3, 2 * wave);
      tp_k3<EL>(lds, lb, q, n, wp, wp, bq, fa, fb, acc, lane);
      PSTAMP(160);
#pragma unroll
      for (int p = 0; p < tp::P; ++p)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) pol[p][ct] = tp_pack<EL>(acc[p][ct]);
    }
    f32x4 acc[tp::P][2];
    float4 b4[2];
    tp_bias(b4, a.x.be1, 32 * wave, q);
    tp_init<EL, 0>(acc, b4, 32 * wave, res[0], nullptr, 0, 0, q);
    tp_pin(acc);
    tp_k1<EL>(lds, lb, q, n, tpw1(a.x.we1, 2 * wave), acc, lane);
    PSTAMP(161);
    __syncthreads();
#pragma unroll
    for (int p = 0; p < tp::P; ++p)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        *reinterpret_cast<uint2*>(lds + p * tp::PIX + tp_cofs(32 * wave + 16 * ct + 4 * q, n)) = pol[p][ct];
        *reinterpret_cast<uint2*>(lds + p * tp::PIX + tp_cofs(128 + 32 * wave + 16 * ct + 4 * q, n)) = tp_pack<EL>(acc[p][ct]);
      }
    __syncthreads();
    const int ntab = a.tree.S + 1;
    const bool tab_lds = a.tree_on && ntab <= tp::NT;
    float tsq = 0.f, tct = 0.f;
    if (tab_lds && tid < ntab) { tsq = a.tree.sqrt_tab[tid]; tct = a.tree.c_tab[tid]; }
    const int hc0[2] = {0, 128}, kind[2] = {0, 1};
    PSTAMP(162);
    tp_heads<EL, 2, 128, 128>(a, lds, hc0, kind, env0, nenv, tid);
    PSTAMP(163);
    if (a.tree_on) {  // this simulation's backup and the next selection (mcts.py:136-234), per env
      float* sc = reinterpret_cast<float*>(lds);
      float* tab = sc + TPH_TAB;
      if (tab_lds && tid < ntab) { tab[tid] = tsq; tab[ntab + tid] = tct; }
      __syncthreads();
      const float* dec = sc + TPH_DEC;
      if (tid < nenv) {
        const int b = env0 + tid;
        tree_backup_env(a.tree, a.tree_sim, b, a.tree_r[b], dec[(16 + tid) * 4], dec + tid * 4, a.tree_gamma);
        if (a.tree_sim + 1 < a.tree.S)
          tree_select_env(a.tree, a.tree_sim + 1, b, tab_lds ? tab : nullptr, tab_lds ? tab + ntab : nullptr);
      }
    }
    PSTAMP(164);
#ifdef TOWERP_STAMPS
    pstamp(PST_N - 2, true);
    pstamp(PST_N - 1);
#endif
    return;
  }
  // the tower output, env-contiguous
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
    const int e = 4 * wave + bb;
    if (e < nenv) {
#pragma unroll
      for (int u = 0; u < 10; ++u) {
        const int cj = u * 64 + lane;
        *reinterpret_cast<uint4*>(a.out + (long long)(env0 + e) * tp::P * tp::C + (long long)cj * 8) =
            Elt<EL>::to_bf16(*reinterpret_cast<const uint4*>(lds + tp::off((cj >> 5) * tp::E + e, cj & 31)));
      }
    }
  }
#ifdef TOWERP_STAMPS
  pstamp(PST_N - 2, true);
  pstamp(PST_N - 1);
#endif
}

}  // namespace

extern "C" {

#ifdef TOWERP_STAMPS
int mzba_towerp_stamps_read(unsigned long long* host, int nrows) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mz_towerp_stamps), sizeof(unsigned long long) * PST_N * nrows);
}
#endif

// Dynamics / prediction step (or the plain tower, epilogue 0) on the pixel-tiled kernel: the
// arguments of mzba_tower_fused (include/mzba.h); bf16 only (x.elem 0). Called by mzba_tower /
// mzba_tower_fused for plan 4, or directly.
int mzba_towerp_fused(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                      void* out, const void* wf16, const float* bias, int nblocks, int B, const mzba_tower_ext* ext,
                      hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && nblocks >= 1 && in && wf16 && bias && ext, -1);
  const mzba_tower_ext& x = *ext;
  MZ_CHECK_ARG((x.elem == 0 || x.elem == 1) && x.epilogue >= 0 && x.epilogue <= 2, -2);
  MZ_CHECK_ARG(!x.w0 || (x.b0 && x.act_bias && x.act && x.A > 0), -3);
  MZ_CHECK_ARG(x.epilogue != 0 || out, -3);
  MZ_CHECK_ARG(x.epilogue != 1 || ((out || x.pool) && x.we1 && x.be1 && x.lw[0] && x.lb[0] && x.dec[0] && x.lO[0] > 1 &&
                                   x.lO[0] <= 16), -3);
  MZ_CHECK_ARG(x.epilogue != 2 || (x.we3 && x.be3 && x.we1 && x.be1 && x.lw[0] && x.lw[1] && x.lb[0] && x.lb[1] &&
                                   x.dec[0] && x.dec[1] && x.lO[0] >= 1 && x.lO[0] <= 16 && x.lO[1] > 1 &&
                                   x.lO[1] <= 16), -3);
  TPArgs a{(const bf16_t*)in, in_env_stride, slot, in_slot_stride, (bf16_t*)out, (const bf16_t*)wf16, bias, nblocks, B,
           x, TreeArgs{}, 0, 0, 0.f, nullptr};
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
  if (x.elem == 1)
    hipLaunchKernelGGL(towerp_kernel<1>, dim3((B + tp::E - 1) / tp::E), dim3(tp::NT), 0, stream, a);
  else
    hipLaunchKernelGGL(towerp_kernel<0>, dim3((B + tp::E - 1) / tp::E), dim3(tp::NT), 0, stream, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

// plain pixel-tiled tower (the arguments of mzba_tower without the workspace)
int mzba_towerp(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride, void* out,
                const void* wf16, const float* bias, int nblocks, int B, hipStream_t stream) {
  mzba_tower_ext x{};
  return mzba_towerp_fused(in, in_env_stride, slot, in_slot_stride, out, wf16, bias, nblocks, B, &x, stream);
}

}  // extern "C"
