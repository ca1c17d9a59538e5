// f16 storage for the 16-bit conv body (nsm_conv_s16.inc), included inside
// namespace nsm_h right before the body's second inclusion: these
// declarations shadow nsm's bf16 helpers of the same names for that copy
// (unqualified lookup stops at the innermost namespace that declares a name;
// none of them takes an argument of an nsm type, so no nsm overload joins by
// argument-dependent lookup),
// so the body's loaders, prologues and epilogues read and write IEEE half and
// its MFMAs run v_mfma_f32_*_f16. Values are rounded to nearest even; beyond
// 65504 they become +-Inf, as under the reference's fp16 autocast.
// Not a header of its own: no include guard, no includes.

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf_lo(uint32_t w) { return (float)__builtin_bit_cast(f16x2, w).x; }
__device__ __forceinline__ float bf_hi(uint32_t w) { return (float)__builtin_bit_cast(f16x2, w).y; }
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) { return pack_h2(f32x2{a, b}); }
__device__ __forceinline__ float round_bf(float a) { return (float)(_Float16)a; }
__device__ __forceinline__ bf16_t s16_bits(float v) { return (bf16_t)(pack_h2(f32x2{v, 0.f}) & 0xFFFFu); }

__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t* p) { return bf_lo((uint32_t)*p); }
__device__ __forceinline__ F8 ld8(const float* p) { return nsm::ld8(p); }
__device__ __forceinline__ F8 ld8(const bf16_t* p) {
  const u32x4 w = *(const u32x4*)p;
  return F8{f32x4{bf_lo(w.x), bf_hi(w.x), bf_lo(w.y), bf_hi(w.y)},
            f32x4{bf_lo(w.z), bf_hi(w.z), bf_lo(w.w), bf_hi(w.w)}};
}
__device__ __forceinline__ void st8s(bf16_t* p, F8 v) {
  *(u32x4*)p = u32x4{pack_bf2(v.a.x, v.a.y), pack_bf2(v.a.z, v.a.w), pack_bf2(v.b.x, v.b.y),
                     pack_bf2(v.b.z, v.b.w)};
}

__device__ __forceinline__ f32x16 mfma_s16_32(bf16x8 a, bf16x8 b, f32x16 c, int, int, int) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_s16_16(bf16x8 a, bf16x8 b, f32x4 c, int, int, int) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
