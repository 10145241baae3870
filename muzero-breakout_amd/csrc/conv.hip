// Implicit-GEMM convolution for the MuZero ResNets on gfx950 MFMA.
//
// out[m][n] = act( sum_k A[m][k] * Wp[n][k] + bias[n] (+ act_bias[p][a_b][n]) (+ res[m][n]) )
//   m = (env b, pixel p = y*W + x)  — NHWC activations, channel stride Cin (multiple of 4 f32 / 8 bf16)
//   k = (tap (ky,kx), channel c)    — A[m][k] = in[b][y+ky-pad][x+kx-pad][c] or 0 (zero padding)
//   Wp[n][k] = BN-folded weights packed K-contiguous per output channel
// One kernel covers every conv of the reference nets (networks.py:7-35, 38-241): 3x3 and
// 1x1, BN folded into (Wp, bias) on the host, ReLU and the residual add fused into the
// epilogue, and the dynamics net's one-hot action planes folded into a per-(pixel, action)
// bias table (mcts.py:252-268 planes are constant over the grid, so their conv
// contribution only depends on the pixel's in-bounds taps).
//
// Tile 128x128, 4 waves (2x2), each wave 64x64 = 4x4 MFMA 16x16 tiles. One K-step moves
// one 128-byte row slice per tile row (BK = 64 bf16 or 32 f32), split into
// tap-resolved 16-B chunks (Cin % 4 f32 / % 8 bf16). Operands staged global -> VGPR -> LDS (double buffer, one barrier
// per K-step), 16-B chunks XOR-swizzled by (row & 7) so the fragment reads are spread
// over the LDS banks. bf16 uses v_mfma_f32_16x16x32_bf16; the f32 parity path uses
// v_mfma_f32_16x16x4_f32 (exact f32 fma chain).
#include "common.h"
#include <type_traits>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 128, BN = 128, NT = 256;
constexpr int ROWB = 128;  // bytes per tile row per K-step

struct ConvArgs {
  const void* in;
  long long in_env_stride;   // elements between consecutive envs of the input
  long long in_slot_stride;  // elements between node slots (latent pool); used when slot != null
  const int32_t* slot;       // optional per-env slot index (gather of parent latents)
  const void* w;             // [Cout][taps*Cin]
  const float* bias;         // [Cout]
  const float* act_bias;     // optional [HW][A][Cout]
  const int32_t* act;        // optional per-env action
  int A;
  const void* res;           // optional residual, [B*HW][Cout]
  void* out;                 // [B*HW][Cout]
  int B, H, W, Cin, Cout, ks, relu;
};

template <typename T> struct Tr;
template <> struct Tr<bf16_t> { static constexpr int BK = 64; };
template <> struct Tr<float> { static constexpr int BK = 32; };

MZ_DEV int swz(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 7)) << 4); }

template <typename T>
__global__ __launch_bounds__(NT, 2) void conv_igemm_kernel(ConvArgs a) {
  constexpr int BK = Tr<T>::BK;
  constexpr int EPC = 16 / sizeof(T);  // elements per 16-B chunk
  __shared__ __attribute__((aligned(16))) uint8_t lds[2][2][BM * ROWB];  // [buf][A/B]
  const int HW = a.H * a.W;
  const int M = a.B * HW;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int pad = a.ks / 2;
  const int Ktot = a.ks * a.ks * a.Cin;
  const int nK = (Ktot + BK - 1) / BK;  // the last K-step may be ragged (zero-filled)

  // per-thread staging geometry: chunk j of rows r + 32*i
  const int j = tid & 7, r0 = tid >> 3;
  const T* in = (const T*)a.in;
  const T* wgt = (const T*)a.w;
  const T* abase[4];
  int ay[4], ax[4];
  bool mval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = m0 + r0 + 32 * i;
    mval[i] = m < M;
    int mm = mval[i] ? m : 0;
    int b = mm / HW, p = mm - b * HW;
    ay[i] = p / a.W; ax[i] = p - ay[i] * a.W;
    long long off = (long long)b * a.in_env_stride;
    if (a.slot) off += (long long)a.slot[b] * a.in_slot_stride;
    abase[i] = in + off;
  }

  uint4 ra[4], rb[4];
  bool oka[4], okb[4];
  // each 16-B chunk j of a K-step resolves its own tap (Cin % EPC == 0: a chunk never
  // straddles two taps), so Cin need not be a multiple of BK
  auto load_tile = [&](int ks) {
    const int k = ks * BK + j * EPC;
    const bool kok = k < Ktot;
    const int tap = k / a.Cin, c = k - tap * a.Cin;
    const int ky = tap / a.ks - pad, kx = tap % a.ks - pad;
    // unconditional loads from a clamped (valid) address; the zero select happens at the LDS
    // store (store_tile), after the MFMAs: hipcc waits for a load under a branch inside the
    // branch, which serialised the 8 loads of a K-step and exposed their latency
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int sy = ay[i] + ky, sx = ax[i] + kx;
      oka[i] = kok && mval[i] && sy >= 0 && sy < a.H && sx >= 0 && sx < a.W;
      ra[i] = *reinterpret_cast<const uint4*>(abase[i] + (oka[i] ? (long long)(sy * a.W + sx) * a.Cin + c : 0));
      int n = n0 + r0 + 32 * i;
      okb[i] = kok && n < a.Cout;
      rb[i] = *reinterpret_cast<const uint4*>(wgt + (okb[i] ? (long long)n * Ktot + k : 0));
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row = r0 + 32 * i;
      *reinterpret_cast<uint4*>(&lds[buf][0][swz(row, j)]) = oka[i] ? ra[i] : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(&lds[buf][1][swz(row, j)]) = okb[i] ? rb[i] : make_uint4(0, 0, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int ks = 0; ks < nK; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nK) load_tile(ks + 1);
    const uint8_t* la = lds[buf][0];
    const uint8_t* lb = lds[buf][1];
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[4], bfv[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          int row = wm * 64 + mi * 16 + fr;
          af[mi] = *reinterpret_cast<const bf16x8*>(la + swz(row, kk * 4 + fq));
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          int row = wn * 64 + ni * 16 + fr;
          bfv[ni] = *reinterpret_cast<const bf16x8*>(lb + swz(row, kk * 4 + fq));
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfv[ni], acc[mi][ni], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) {
        float af[4], bfv[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          int row = wm * 64 + mi * 16 + fr;
          af[mi] = *reinterpret_cast<const float*>(la + swz(row, kc) + fq * 4);
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          int row = wn * 64 + ni * 16 + fr;
          bfv[ni] = *reinterpret_cast<const float*>(lb + swz(row, kc) + fq * 4);
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mi], bfv[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    if (ks + 1 < nK) store_tile(buf ^ 1);
    __syncthreads();
  }

  // epilogue: D[row = 4*fq + r][col = fr] of each 16x16 tile. Per channel tile, every action-bias /
  // residual load of the lane's 16 outputs is issued (from clamped addresses) before the first use,
  // op order unchanged ((((acc + act_bias) + bias) + res), ReLU): the per-element form waited one
  // memory round trip per output (two with the action index), 64 per lane.
  T* out = (T*)a.out;
  const T* res = (const T*)a.res;
  int mrow[4][4], arow[4][4];  // [mi][r]: pixel row (clamped), action-bias row p * A + act[env]
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) mrow[mi][r] = min(m0 + wm * 64 + mi * 16 + fq * 4 + r, M - 1);
  if (a.act_bias) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = mrow[mi][r] / HW, p = mrow[mi][r] - b * HW;
        arow[mi][r] = p * a.A + a.act[b];
      }
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + fr;
    const int nc = min(n, a.Cout - 1);
    const float bn = a.bias[nc];
    float ab[4][4], rv[4][4];
    if (a.act_bias) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) ab[mi][r] = a.act_bias[(long long)arow[mi][r] * a.Cout + nc];
    }
    if (res) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) rv[mi][r] = ElemIO<T>::load(res + (long long)mrow[mi][r] * a.Cout + nc);
    }
    if (n >= a.Cout) continue;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + mi * 16 + fq * 4 + r;
        if (m >= M) continue;
        float v = acc[mi][ni][r];
        if (a.act_bias) v = v + ab[mi][r];
        v = v + bn;
        if (res) v = v + rv[mi][r];
        if (a.relu) v = fmaxf(v, 0.f);
        ElemIO<T>::store(out + (long long)m * a.Cout + n, v);
      }
    }
  }
}

// Large-image bf16 conv (config 3 geometry: 84x84 / 42x42 images, 21x21 latents; M = B*H*W in the
// millions): one workgroup = 256 pixels x 256 output channels, 8 waves (2 pixel halves x 4 channel
// quarters, two per SIMD), each 128 x 64 = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 with the WEIGHTS as
// the A operand, so a lane's accumulator holds 4 consecutive channels of one pixel (8-byte bf16
// stores). K step = 64 (one tap, a 64-channel block: Cin % 64 == 0), walked with scalar counters.
// Staging global -> VGPR -> LDS (two LDS stages, one barrier per step), loads from clamped addresses
// with a zero select at the LDS write (out-of-image taps); weights through a buffer resource.
// The epilogue issues every bias / residual load before the first use: the per-element form waited
// for one memory round trip per (pixel tile, channel tile), 32 per workgroup, about as long as the
// whole k loop (+20 % on the 21x21 latent conv, profiles/r02/conv_big/).
namespace big {
constexpr int BM = 256, BN = 256, NT = 512, BK = 64, ROWB = 128;
constexpr int TILE = BM * ROWB;     // 32 KB per operand per stage
constexpr int RPT = BM / (NT / 8);  // staged rows per thread per operand (4)
}

__global__ __launch_bounds__(big::NT, 1) void conv_big_bf16_kernel(ConvArgs a) {
  using big::NT; using big::BK; using big::TILE; using big::RPT;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_big[];  // [2 stages][A | W]
  const int HW = a.H * a.W;
  const int M = a.B * HW;
  const int m0 = blockIdx.x * big::BM, n0 = blockIdx.y * big::BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;  // pixel half (128), channel quarter (64)
  const int pad = a.ks / 2;
  const int Ktot = a.ks * a.ks * a.Cin;  // Cin % 64 == 0 (launcher): a K step lies within one tap
  const int nK = Ktot / BK;
  const int j = tid & 7, r0 = tid >> 3;  // staging: chunk j of rows r0 + 64 i
  // per staged pixel row: its offset in 16-B units (the address every out-of-image tap falls back
  // to) and (y, x) packed
  int aoff[RPT], ayx[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int m = m0 + r0 + 64 * i;
    const int mm = m < M ? m : 0;
    const int bb = mm / HW, p = mm - bb * HW;
    const int y = p / a.W;
    ayx[i] = m < M ? (y << 16) | (p - y * a.W) : 0x7fff7fff;  // invalid rows: no tap in the image
    aoff[i] = (int)(((long long)bb * a.in_env_stride + (long long)p * a.Cin) >> 3);
  }
  const uint4* in16 = reinterpret_cast<const uint4*>(a.in) + j;
  // weights through a buffer resource over this workgroup's 256 rows (Cout % 256 == 0): the lane's
  // row / chunk offset in one VGPR, the row group and K step in the scalar offset
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>((const bf16_t*)a.w + (long long)n0 * Ktot), 0, big::BN * Ktot * 2, 0x00020000);
  const int wvoff = (r0 * Ktot + j * 8) * 2;
  uint4 ra[2][RPT], rb[RPT];
  uint32_t oka[2];
  // walk state of the next activation step (lc, lky, lkx) and the next weight step (lw)
  int lc = 0, lky = -pad, lkx = -pad, lw = 0;
  auto load_a = [&](auto setc) {
    constexpr int set = decltype(setc)::value;
    const int toff = ((lky * a.W + lkx) * a.Cin + lc) >> 3;
    uint32_t ok = 0;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int sy = (ayx[i] >> 16) + lky, sx = (ayx[i] & 0xffff) + lkx;
      const bool o = (unsigned)sy < (unsigned)a.H && (unsigned)sx < (unsigned)a.W;
      ok |= (o ? 1u : 0u) << i;
      ra[set][i] = in16[aoff[i] + (o ? toff : 0)];
    }
    oka[set] = ok;
    lc += BK;
    if (lc == a.Cin) {
      lc = 0;
      if (++lkx > pad) { lkx = -pad; ++lky; }
    }
  };
  auto load_w = [&]() {
#pragma unroll
    for (int i = 0; i < RPT; ++i)
      rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoff, (64 * i * Ktot + lw) * 2, 0));
    lw += BK;
  };
  auto store_tile = [&](auto setc, int buf) {
    constexpr int set = decltype(setc)::value;
    uint8_t* la = lds_big + buf * 2 * TILE;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int row = r0 + 64 * i;
      *reinterpret_cast<uint4*>(la + swz(row, j)) = ((oka[set] >> i) & 1) ? ra[set][i] : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(la + TILE + swz(row, j)) = rb[i];
    }
  };
  f32x4 acc[8][4];  // [pixel tile][channel tile]: D[channel 4q + i][pixel l16]
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  load_a(std::integral_constant<int, 0>{});
  load_w();
  if (nK > 1) load_a(std::integral_constant<int, 1>{});
  store_tile(std::integral_constant<int, 0>{}, 0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  // one K step on LDS stage SET; activation register set SET was written at the end of the previous
  // step and is refilled with step ks + 2; the weight set with step ks + 1. (The compiler's wait
  // counting merges the paths of the two conditions and waits for every older load before these are
  // issued: in effect one step of lead, as before; a branch-free form of the loop spills.)
  auto step = [&](int ks, auto setc) {
    constexpr int SET = decltype(setc)::value;
    if (ks + 2 < nK) load_a(setc);
    if (ks + 1 < nK) load_w();
    const uint8_t* la = lds_big + SET * 2 * TILE;
    const uint8_t* lwt = la + TILE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 wf[4], xf[8];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        wf[ni] = *reinterpret_cast<const bf16x8*>(lwt + swz(wn * 64 + ni * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
        xf[mi] = *reinterpret_cast<const bf16x8*>(la + swz(wm * 128 + mi * 16 + fr, kk * 4 + fq));
      __builtin_amdgcn_s_setprio(1);  // keep the MFMA cluster together (cdna_hip_programming T5)
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], xf[mi], acc[mi][ni], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (ks + 1 < nK) store_tile(std::integral_constant<int, 1 - SET>{}, 1 - SET);
    __syncthreads();
  };
  for (int ks = 0; ks < nK; ks += 2) {
    step(ks, std::integral_constant<int, 0>{});
    if (ks + 1 < nK) step(ks + 1, std::integral_constant<int, 1>{});
  }
  // epilogue: lane holds channels n .. n+3 of pixel m: + bias (+ residual), ReLU, 8-byte stores.
  // Every bias / residual load is issued (from clamped rows) before the first use: written per
  // element (load, add, store) the compiler waited vmcnt(0) 32 times per workgroup, one round trip
  // each (as long as the whole k loop).
  bf16_t* out = (bf16_t*)a.out;
  const bf16_t* res = (const bf16_t*)a.res;
  float4 bb[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) bb[ni] = *reinterpret_cast<const float4*>(a.bias + n0 + wn * 64 + ni * 16 + 4 * fq);
  uint2 rv[8][4];
  if (res) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = min(m0 + wm * 128 + mi * 16 + fr, M - 1);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        rv[mi][ni] = *reinterpret_cast<const uint2*>(res + (long long)m * a.Cout + n0 + wn * 64 + ni * 16 + 4 * fq);
    }
  } else {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) rv[mi][ni] = make_uint2(0x80008000u, 0x80008000u);  // bf16 -0
  }
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int m = m0 + wm * 128 + mi * 16 + fr;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int n = n0 + wn * 64 + ni * 16 + 4 * fq;
      const uint2 r = rv[mi][ni];
      // (acc + bias) + residual: the residual-free form adds -0, which leaves every value (and the
      // sign of a zero) unchanged
      float v0 = (acc[mi][ni][0] + bb[ni].x) + bf16_to_f32((bf16_t)(r.x & 0xffffu));
      float v1 = (acc[mi][ni][1] + bb[ni].y) + bf16_to_f32((bf16_t)(r.x >> 16));
      float v2 = (acc[mi][ni][2] + bb[ni].z) + bf16_to_f32((bf16_t)(r.y & 0xffffu));
      float v3 = (acc[mi][ni][3] + bb[ni].w) + bf16_to_f32((bf16_t)(r.y >> 16));
      if (a.relu) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
      if (m < M)
        *reinterpret_cast<uint2*>(out + (long long)m * a.Cout + n) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    }
  }
}

// 2x2 average pool, NHWC (networks.py:44 nn.AvgPool2d(2, 2))
template <typename T>
__global__ void avgpool2_kernel(const T* __restrict__ in, T* __restrict__ out, int B, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2;
  size_t n = (size_t)B * Ho * Wo * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    size_t q = i / C;
    int xo = (int)(q % Wo);
    size_t q2 = q / Wo;
    int yo = (int)(q2 % Ho);
    size_t b = q2 / Ho;
    const T* base = in + ((b * H + 2 * yo) * W + 2 * xo) * C + c;
    float s = ElemIO<T>::load(base) + ElemIO<T>::load(base + C);
    s = s + ElemIO<T>::load(base + (size_t)W * C);
    s = s + ElemIO<T>::load(base + (size_t)W * C + C);
    ElemIO<T>::store(out + i, s / 4.0f);
  }
}

// per-env min-max scaling (networks.py:314-328) over the HW*C values: one wave per env, a
// single pass (the env's values stay in registers between the min/max and the write), 16-B
// accesses. Writes the scaled latent to out and, when pool != null, to its node-pool slot.
template <typename T, int CPL>
__global__ __launch_bounds__(256) void scale_state_kernel(const T* __restrict__ h, T* __restrict__ out,
                                                          T* __restrict__ pool, long long pool_env_stride,
                                                          const int32_t* __restrict__ slot_arr, int slot_const,
                                                          long long slot_stride, int B, int n) {
  constexpr int EPC = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int nch = n / EPC;
  const uint4* x = reinterpret_cast<const uint4*>(h + (size_t)b * n);
  uint4 v[CPL];
  float mn = INFINITY, mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < CPL; ++u) {
    const int c = u * 64 + lane;
    v[u] = c < nch ? x[c] : x[0];
    const T* e = reinterpret_cast<const T*>(&v[u]);
#pragma unroll
    for (int j = 0; j < EPC; ++j) {
      const float f = ElemIO<T>::load(e + j);
      mn = fminf(mn, f); mx = fmaxf(mx, f);
    }
  }
  for (int o = 32; o > 0; o >>= 1) { mn = fminf(mn, __shfl_xor(mn, o)); mx = fmaxf(mx, __shfl_xor(mx, o)); }
  const float den = (mx - mn) + 1e-8f;
  uint4* o1 = reinterpret_cast<uint4*>(out + (size_t)b * n);
  uint4* o2 = nullptr;
  if (pool) {
    const int s = slot_arr ? slot_arr[b] : slot_const;
    o2 = reinterpret_cast<uint4*>(pool + (size_t)b * pool_env_stride + (size_t)s * slot_stride);
  }
#pragma unroll
  for (int u = 0; u < CPL; ++u) {
    const int c = u * 64 + lane;
    if (c >= nch) break;
    uint4 r = v[u];
    T* e = reinterpret_cast<T*>(&r);
#pragma unroll
    for (int j = 0; j < EPC; ++j) ElemIO<T>::store(e + j, (ElemIO<T>::load(e + j) - mn) / den);
    o1[c] = r;
    if (o2) o2[c] = r;
  }
}

// generic two-pass fallback for large latents (e.g. 21x21x256 at 84x84): one workgroup per env
template <typename T>
__global__ __launch_bounds__(256) void scale_state_big_kernel(const T* __restrict__ h, T* __restrict__ out,
                                                              T* __restrict__ pool, long long pool_env_stride,
                                                              const int32_t* __restrict__ slot_arr, int slot_const,
                                                              long long slot_stride, int n) {
  const int b = blockIdx.x;
  const T* x = h + (size_t)b * n;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = ElemIO<T>::load(x + i);
    mn = fminf(mn, v); mx = fmaxf(mx, v);
  }
  for (int o = 32; o > 0; o >>= 1) { mn = fminf(mn, __shfl_xor(mn, o)); mx = fmaxf(mx, __shfl_xor(mx, o)); }
  __shared__ float smn[4], smx[4];
  if ((threadIdx.x & 63) == 0) { smn[threadIdx.x >> 6] = mn; smx[threadIdx.x >> 6] = mx; }
  __syncthreads();
  mn = fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3]));
  mx = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
  const float den = (mx - mn) + 1e-8f;
  T* o = out + (size_t)b * n;
  T* po = nullptr;
  if (pool) po = pool + (size_t)b * pool_env_stride + (size_t)(slot_arr ? slot_arr[b] : slot_const) * slot_stride;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = (ElemIO<T>::load(x + i) - mn) / den;
    ElemIO<T>::store(o + i, v);
    if (po) ElemIO<T>::store(po + i, v);
  }
}

static thread_local int g_conv_big = 1;  // 1: large bf16 convs on conv_big_bf16_kernel (mzba_conv2d_set_variant)

template <typename T>
int launch_conv(const ConvArgs& a, hipStream_t s) {
  const int M = a.B * a.H * a.W;
  // large images: 256 x 256 tiles (the 4x5 / 8x10 / 16x20 convs have their own kernels)
  // conv_big addresses activation rows in 16-B units with 32-bit offsets
  const bool span32 = ((long long)a.B * a.in_env_stride) / 8 < 0x7fff0000LL;
  if (sizeof(T) == 2 && g_conv_big && a.Cout % 256 == 0 && a.Cin % 64 == 0 && !a.act_bias && !a.slot &&
      M >= 64 * 1024 && span32) {
    static bool attr = false;
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_big_bf16_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 4 * big::TILE);
      if (e != hipSuccess) return (int)e;
      attr = true;
    }
    dim3 grid((M + big::BM - 1) / big::BM, a.Cout / big::BN);
    hipLaunchKernelGGL(conv_big_bf16_kernel, grid, dim3(big::NT), 4 * big::TILE, s, a);
    MZ_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid((M + BM - 1) / BM, (a.Cout + BN - 1) / BN);
  hipLaunchKernelGGL(conv_igemm_kernel<T>, grid, dim3(NT), 0, s, a);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // namespace

extern "C" {

// 1 (default): bf16 convs with M >= 64K pixels, Cout % 256 == 0, no action bias / slot gather on the
// 256 x 256 large-image kernel; 0: always conv_igemm
int mzba_conv2d_set_variant(int v) {
  if (v < 0 || v > 1) return -1;
  g_conv_big = v;
  return 0;
}

// dtype: 0 = f32 (parity), 1 = bf16
int mzba_conv2d(int dtype, const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                const void* w, const float* bias, const float* act_bias, const int32_t* act, int A, const void* res,
                void* out, int B, int H, int W, int Cin, int Cout, int ks, int relu, hipStream_t stream) {
  const int EPC = dtype ? 8 : 4;  // elements per 16-B chunk
  MZ_CHECK_ARG(B > 0 && H > 0 && W > 0 && (ks == 1 || ks == 3), -1);
  MZ_CHECK_ARG(Cin % EPC == 0 && Cout % 4 == 0, -2);
  MZ_CHECK_ARG(!act_bias || (act && A > 0), -3);
  ConvArgs a{in, in_env_stride, in_slot_stride, slot, w, bias, act_bias, act, A, res, out, B, H, W, Cin, Cout, ks, relu};
  return dtype ? launch_conv<bf16_t>(a, stream) : launch_conv<float>(a, stream);
}

int mzba_avgpool2(int dtype, const void* in, void* out, int B, int H, int W, int C, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && H >= 2 && W >= 2, -1);
  size_t n = (size_t)B * (H / 2) * (W / 2) * C;
  unsigned grid = (unsigned)((n + 255) / 256);
  if (grid > 8192) grid = 8192;
  if (dtype)
    hipLaunchKernelGGL(avgpool2_kernel<bf16_t>, dim3(grid), dim3(256), 0, stream, (const bf16_t*)in, (bf16_t*)out, B,
                       H, W, C);
  else
    hipLaunchKernelGGL(avgpool2_kernel<float>, dim3(grid), dim3(256), 0, stream, (const float*)in, (float*)out, B, H,
                       W, C);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_scale_state(int dtype, const void* h, void* out, void* pool, long long pool_env_stride,
                     const int32_t* slot_arr, int slot_const, long long slot_stride, int B, int n,
                     hipStream_t stream) {
  const int epc = dtype ? 8 : 4;
  MZ_CHECK_ARG(B > 0 && n > 0, -1);
  if (n % epc != 0 || n / epc > 64 * (dtype ? 10 : 20)) {
    if (dtype)
      hipLaunchKernelGGL(scale_state_big_kernel<bf16_t>, dim3(B), dim3(256), 0, stream, (const bf16_t*)h,
                         (bf16_t*)out, (bf16_t*)pool, pool_env_stride, slot_arr, slot_const, slot_stride, n);
    else
      hipLaunchKernelGGL(scale_state_big_kernel<float>, dim3(B), dim3(256), 0, stream, (const float*)h, (float*)out,
                         (float*)pool, pool_env_stride, slot_arr, slot_const, slot_stride, n);
    MZ_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid((B + 3) / 4);
  if (dtype)
    hipLaunchKernelGGL((scale_state_kernel<bf16_t, 10>), grid, dim3(256), 0, stream, (const bf16_t*)h, (bf16_t*)out,
                       (bf16_t*)pool, pool_env_stride, slot_arr, slot_const, slot_stride, B, n);
  else
    hipLaunchKernelGGL((scale_state_kernel<float, 20>), grid, dim3(256), 0, stream, (const float*)h, (float*)out,
                       (float*)pool, pool_env_stride, slot_arr, slot_const, slot_stride, B, n);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
