// Element types of the tower kernels' LDS images and weights (tower.hip, towerp.hip).
#pragma once
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// Element type of the LDS images and weights: EL 0 = bf16, 1 = fp16 (the fp16 dynamics net of
// BASELINE config 5). Latents in HBM (tower input, node pool, output) stay bf16: fp16 towers
// convert on staging and write the scaled latent back as bf16.
template <int EL> struct Elt;
template <> struct Elt<0> {
  typedef bf16x8 v8;
  static MZ_DEV f32x4 mfma(v8 a, v8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
  static MZ_DEV uint32_t pack2(float a, float b) { return pack_bf16x2(a, b); }
  static MZ_DEV float lo(uint32_t u) { return __uint_as_float(u << 16); }
  static MZ_DEV float hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
  static MZ_DEV uint4 from_bf16(uint4 v) { return v; }
  static MZ_DEV uint4 to_bf16(uint4 v) { return v; }
};
template <> struct Elt<1> {
  typedef f16x8 v8;
  static MZ_DEV f32x4 mfma(v8 a, v8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
  static MZ_DEV uint32_t pack2(float a, float b) {
    const f16x2 v = {(_Float16)a, (_Float16)b};  // round to nearest even
    return __builtin_bit_cast(uint32_t, v);
  }
  static MZ_DEV float lo(uint32_t u) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu)); }
  static MZ_DEV float hi(uint32_t u) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16)); }
  static MZ_DEV uint4 from_bf16(uint4 v) {
    return make_uint4(pack2(Elt<0>::lo(v.x), Elt<0>::hi(v.x)), pack2(Elt<0>::lo(v.y), Elt<0>::hi(v.y)),
                      pack2(Elt<0>::lo(v.z), Elt<0>::hi(v.z)), pack2(Elt<0>::lo(v.w), Elt<0>::hi(v.w)));
  }
  static MZ_DEV uint4 to_bf16(uint4 v) {
    return make_uint4(pack_bf16x2(lo(v.x), hi(v.x)), pack_bf16x2(lo(v.y), hi(v.y)), pack_bf16x2(lo(v.z), hi(v.z)),
                      pack_bf16x2(lo(v.w), hi(v.w)));
  }
};
// the 8 values of a 16-B chunk of element type EL as f32
template <int EL> MZ_DEV void unpack8(uint4 v, float (&f)[8]) {
  f[0] = Elt<EL>::lo(v.x); f[1] = Elt<EL>::hi(v.x); f[2] = Elt<EL>::lo(v.y); f[3] = Elt<EL>::hi(v.y);
  f[4] = Elt<EL>::lo(v.z); f[5] = Elt<EL>::hi(v.z); f[6] = Elt<EL>::lo(v.w); f[7] = Elt<EL>::hi(v.w);
}

}  // namespace
