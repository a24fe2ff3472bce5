// MFMA policies for the two compute precisions of the hfrep kernels (gfx950 only).
//
//   bf16 storage  -> v_mfma_f32_32x32x16_bf16   (K step 16, 8 bf16 per lane per operand)
//   fp32 storage  -> v_mfma_f32_32x32x2_f32     (K step 2, exact fp32 fmaf chain)
//
// Both produce the same 32x32 fp32 accumulator layout (col = lane&31,
// row = (r&3) + 8*(r>>2) + 4*(lane>>5)), so every kernel is written once over a policy.
// Operand lane maps (CDNA4 guide §3):
//   32x32x16 bf16: lane l holds A[l&31][8*(l>>5) + j] and B[8*(l>>5) + j][l&31], j = 0..7
//   32x32x2  f32 : lane l holds A[l&31][l>>5]         and B[l>>5][l&31]
#pragma once
#include "common.h"

namespace hfrep {

template <typename T> struct MF;

template <> struct MF<float> {
  static constexpr int KS = 2;
  static constexpr int LDS_PAD = 1;  // row pad (elements) that makes ds_read_b32 column reads conflict-free
  typedef float frag;
  __device__ __forceinline__ static frag zero() { return 0.f; }
  // A fragment from an LDS row that holds this lane's matrix row (k contiguous)
  __device__ __forceinline__ static frag lda(const float* row, int ks, int lane) { return row[ks * 2 + (lane >> 5)]; }
  // B fragment built element-wise from a functor get(k) for this lane's column
  template <class G> __device__ __forceinline__ static frag make(G get, int ks, int lane) {
    return get(ks * 2 + (lane >> 5));
  }
  __device__ __forceinline__ static f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
};

template <> struct MF<bf16_t> {
  static constexpr int KS = 16;
  static constexpr int LDS_PAD = 8;  // keeps 16-B alignment and spreads ds_read_b128 over banks
  typedef bf16x8 frag;
  __device__ __forceinline__ static frag zero() { return frag{0, 0, 0, 0, 0, 0, 0, 0}; }
  __device__ __forceinline__ static frag lda(const bf16_t* row, int ks, int lane) {
    return *reinterpret_cast<const bf16x8*>(row + ks * 16 + 8 * (lane >> 5));
  }
  template <class G> __device__ __forceinline__ static frag make(G get, int ks, int lane) {
    frag f;
    const int k0 = ks * 16 + 8 * (lane >> 5);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (short)f2bf(get(k0 + j));
    return f;
  }
  __device__ __forceinline__ static f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

}  // namespace hfrep
