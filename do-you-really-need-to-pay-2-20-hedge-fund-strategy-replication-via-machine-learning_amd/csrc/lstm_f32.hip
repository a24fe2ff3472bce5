// fp32 LSTM layer kernels (gfx950): exact-fp32 MFMA, fused input projection, persistent.
//
// The fp32 (reference-precision) path used to run the v1 recurrences of lstm.hip on a zx = x W + b
// tensor materialised by a separate GEMM: at B = 32k that GEMM alone wrote 1.3 GB per layer call and
// the v1 recurrence issued its zx loads at the top of every step (profiles/r02_prof_fp32: the
// linear / wgrad GEMMs were 60 % and the recurrences 37 % of the fp32 step).  In fp32 the matrix
// pipe is the bound (v_mfma_f32_16x16x4_f32: 64 FLOP/clk/SIMD, 1/16 of bf16), so this design is
// about keeping MFMA issue dense and the padding small:
//
//  * 4 waves per workgroup, ONE per SIMD (~400 VGPRs each), one persistent workgroup per CU walking
//    32-row tiles.  Wave w owns units 28 w .. 28 w + 27 (100 units -> 7 + 7 + 7 + 4 tiles of 4 units;
//    12 % padding instead of the 28 % of 32-unit waves);
//  * GATE-INTERLEAVED 16-column MFMA tiles: column c of tile n is gate (c & 3) of unit
//    28 w + 4 n + (c >> 2), so the four gates of a unit sit in one lane quad.  Each lane applies
//    its own gate's nonlinearity to its 4 accumulator rows (no lane computes a gate it does not
//    own), then a 4 x 4 quad transpose (DPP quad_perm) gives every lane the i, f, g, o of ONE
//    (row, unit) for the cell update: no redundant transcendentals and a 1-register cell state;
//  * U^T fragments in registers (25 k-steps x 7 tiles), W^T fragments in registers for the first
//    12 k-steps and in LDS for the rest (K = 100: 93 KB), so z_t = x_t W + h_{t-1} U + b is one
//    MFMA chain per tile and zx never exists in HBM;
//  * A operands (x_t, h_{t-1}) in LDS in a K-permuted layout (element k at (k & 3) * KQ + (k >> 2)
//    of its row) so one ds_read_b128 feeds four 16x16x4 k-steps; the row strides are chosen
//    conflict-free for ds_read_b128 (scripted search over the CDNA4 lane groups);
//  * x_{t+1} is loaded into registers at the top of step t and written to LDS at its end, so its
//    HBM latency hides under the step's ~700 MFMAs;
//  * outputs in the row-major layouts of the v1 contract (h (B,T,H), gate activations (B,T,4H),
//    cells (B,T,H); the tangent's hdot, zdot, cdot), so the v1 reverse kernels consume them.
//
// TAN = true is the tangent forward at a saved primal point (ops/reference.py lstm_seq_tfwd with
// dzx = xd W folded in): zdot_t = xd_t W + hdot_{t-1} U, primal gates / cells read from the tape.
#include "common.h"
#include "kernels.h"

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <set>
#include <stdexcept>

namespace hfrep {

namespace {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef int v4i_t __attribute__((ext_vector_type(4)));
constexpr int kOOB = 0x7fff0000;  // voffset past every descriptor's num_records (see lstm2.hip)

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
// rows [row0, row0 + 32) (clipped to B) of a row-major (B, Tn, W) fp32 tensor
__device__ __forceinline__ rsrc_t ftile_rsrc(const float* base, int row0, int B, int Tn, int W) {
  row0 = __builtin_amdgcn_readfirstlane(row0);
  const int nr = base ? max(0, min(32, B - row0)) : 0;
  return make_rsrc(base + (nr ? (size_t)row0 * Tn * W : 0), nr * Tn * W * 4);
}
__device__ __forceinline__ float ld1(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ void st1(float v, rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, voff, soff, 0);
}

// geometry of a K-wide A operand tile (32 rows) in LDS: KS k-steps of 4; element k of a row at
// (k & 3) * KQ + (k >> 2); row stride LR.  (KQ, LR) = (12, 56) / (28, 120) are conflict-free for the
// ds_read_b128 fragment reads (lane l: row l & 15, k-group l >> 4) over all four lane groups.
template <int K>
struct FGeo {
  static_assert(K >= 1 && K <= 112, "fp32 LSTM: K <= 112");
  static constexpr int KS = (K + 3) / 4;
  static constexpr int KQ = KS <= 12 ? 12 : 28;
  static constexpr int LR = KS <= 12 ? 56 : 120;
  static constexpr int NJ = (KS + 3) / 4;  // b128 reads per row
};
constexpr int FH = 100, FG = 400, FNT = 7, FUW = 28;
// W^T k-steps kept in registers (the rest live in LDS)
template <int K>
constexpr int f_nwr() { return FGeo<K>::KS <= 12 ? FGeo<K>::KS : 12; }
template <int K>
constexpr int f_nwl() { return FGeo<K>::KS - f_nwr<K>(); }

__device__ __forceinline__ f32x4 mma4(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// quad_perm DPP moves (lane q of each quad reads lane perm[q])
__device__ __forceinline__ float qswap2(float v) {  // [2,3,0,1]
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
}
__device__ __forceinline__ float qswap1(float v) {  // [1,0,3,2]
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
}
// 4 x 4 transpose inside each lane quad: lane q holds a[i] = M[q][i]; afterwards a[k] = M[k][q]
__device__ __forceinline__ void quad_transpose(float (&a)[4], int q) {
  const float p0 = qswap2(a[0]), p1 = qswap2(a[1]), p2 = qswap2(a[2]), p3 = qswap2(a[3]);
  const bool lo = q < 2;
  const float b0 = lo ? a[0] : p2, b1 = lo ? a[1] : p3, b2 = lo ? p0 : a[2], b3 = lo ? p1 : a[3];
  const float r0 = qswap1(b0), r1 = qswap1(b1), r2 = qswap1(b2), r3 = qswap1(b3);
  const bool ev = !(q & 1);
  a[0] = ev ? b0 : r1;
  a[1] = ev ? r0 : b1;
  a[2] = ev ? b2 : r3;
  a[3] = ev ? r2 : b3;
}

// x tile loader: this thread's share of the 32 x K tile of one step, loaded to registers and
// written to the K-permuted LDS layout.  Offsets are computed once per row block.
template <int K>
struct FXPart {
  static constexpr bool VEC = K % 4 == 0;
  static constexpr int PER = VEC ? K / 4 : K;                 // chunks per row
  static constexpr int NJ = (32 * PER + 255) / 256;
  float v[VEC ? 4 * NJ : NJ];
  int goff[NJ], lpos[NJ];
  __device__ __forceinline__ void set(int Tn, int tid) {
    using GX = FGeo<K>;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int e = tid + 256 * j, r = e / PER, c = e - r * PER;
      const bool ok = r < 32;
      if constexpr (VEC) {
        goff[j] = ok ? (r * Tn * K + 4 * c) * 4 : kOOB;
        lpos[j] = ok ? r * GX::LR + c : -1;
      } else {
        goff[j] = ok ? (r * Tn * K + c) * 4 : kOOB;
        lpos[j] = ok ? r * GX::LR + (c & 3) * GX::KQ + (c >> 2) : -1;
      }
    }
  }
  __device__ __forceinline__ void load(rsrc_t rx, int Tn, int t, bool on) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int vo = on ? goff[j] : kOOB;
      if constexpr (VEC) {
        const f32x4 d = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo, t * K * 4, 0));
        v[4 * j] = d[0]; v[4 * j + 1] = d[1]; v[4 * j + 2] = d[2]; v[4 * j + 3] = d[3];
      } else {
        v[j] = ld1(rx, vo, t * K * 4);
      }
    }
  }
  __device__ __forceinline__ void to_lds(float* xb, float* trash) const {
    using GX = FGeo<K>;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float* d = lpos[j] >= 0 ? xb + lpos[j] : trash;
      if constexpr (VEC) {
        const int s = lpos[j] >= 0 ? GX::KQ : 0;
        d[0] = v[4 * j]; d[s] = v[4 * j + 1]; d[2 * s] = v[4 * j + 2]; d[3 * s] = v[4 * j + 3];
      } else {
        d[0] = v[j];
      }
    }
  }
};

// fp32 tape: a lane-native blocked layout.  Per (32-row block, step) and per wave w and accumulator
// pair (m, n) one SLOT of 64 lanes x {4 gate values (16 bytes), 1 cell value}: the lane that computed
// the (row, unit) in the forward reads it back in the reverse kernels, and every wave-level access is
// a contiguous 1 KiB (gates) or 256 B (cell).  Primal tape: gate activations (i, f, g, o) and c_t;
// tangent tape: the gate pre-activation tangents zdot and cdot.  Slots of wave 3's padding tiles
// (units 100..111) are never written nor read.
constexpr int FT_MN = 2 * FNT, FT_SLOT = 64 * 5, FT_STEP = 4 * FT_MN * FT_SLOT;
__device__ __forceinline__ rsrc_t ftape_rsrc(const float* tape, int rb, int nrb, int Tn) {
  rb = __builtin_amdgcn_readfirstlane(rb);
  const bool on = tape && rb < nrb;
  return make_rsrc(tape + (on ? (size_t)rb * Tn * FT_STEP : 0), on ? Tn * FT_STEP * 4 : 0);
}
// byte offset of this lane's gate quad in slot (w, m, n) at step 0; the cell value is at +1024 - 12 lane
__device__ __forceinline__ int ftape_lane(int w, int lane) { return (w * FT_MN * FT_SLOT) * 4 + lane * 16; }
__device__ __forceinline__ int ftape_cell(int w, int lane) { return (w * FT_MN * FT_SLOT + 256 + lane) * 4; }
__device__ __forceinline__ constexpr int ftape_slot(int m, int n) { return (m * FNT + n) * FT_SLOT * 4; }
__device__ __forceinline__ f32x4 ld4(rsrc_t r, int voff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}
__device__ __forceinline__ f32x4 ld4s(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
// one float4 of an X row of XR floats at byte offset voff (+ soff), columns col .. col + 3: one 16-byte
// load when rows are 16-byte aligned; for XR = 35 (the reference's 35 features, staged as a 36-column
// image) four dword loads with the columns >= XR reading zero -- no byte past the row is addressed
template <int XR>
__device__ __forceinline__ f32x4 ldx4(rsrc_t r, int voff, int soff, int col) {
  if constexpr (XR % 4 == 0) {
    return ld4s(r, voff, soff);
  } else {
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff != kOOB && col + i < XR ? voff + 4 * i : kOOB, soff, 0));
    return v;
  }
}
__device__ __forceinline__ void st4(f32x4 v, rsrc_t r, int voff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), r, voff, 0, 0);
}
// 16-byte store at byte offset voff + uoff (uoff uniform) with soffset 0.  A buffer store of more
// than 8 bytes whose data VGPRs the next VALU instruction overwrites needs one wait state, and the
// compiler only inserts it when soffset is NOT a register: with the uniform step offset in soffset
// the BPTT's dZ stores wrote the next value for a few 16-byte chunks per 10^5 rows (rows 14 / 15
// of a 32-row block, r02: profiles/archive_scripts/dbg_large_bwd.py, scripts/isa_store_hazard.py)
__device__ __forceinline__ void st16(f32x4 v, rsrc_t r, bool ok, int voff, int uoff) {
  // (unsigned: voff may already be kOOB; the sum stays past every descriptor's size)
  const int off = (int)((unsigned)voff + (unsigned)uoff);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), r, ok ? off : kOOB, 0, 0);
}

}  // namespace

// ==========================================================================================
// forward / tangent forward
// ==========================================================================================
template <int ACT, int KX, bool TAPE, bool TAN>
__global__ void __launch_bounds__(256, 1)
lstmf_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                 const float* __restrict__ U, const float* __restrict__ ptape, float* __restrict__ hs,
                 float* __restrict__ tape, int B, int Tn) {
  using GX = FGeo<KX>;
  using GH = FGeo<FH>;
  constexpr int NWR = f_nwr<KX>(), NWL = f_nwl<KX>();
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  float* xb = fsm;                     // [2][32 * LRX]
  float* hb = xb + 2 * 32 * GX::LR;    // [2][32 * LRH]
  float* wl = hb + 2 * 32 * GH::LR;    // [NWL][4 waves][7 tiles][64 lanes]
  float* trash = wl + NWL * 4 * FNT * 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane & 3, g = lane >> 4, j4 = (lane & 15) >> 2;
  const int ub = FUW * w + j4;  // unit of tile 0 in this lane's MFMA column; tile n adds 4 n
  const int nrb = (B + 31) / 32;

  for (int i = tid; i < 2 * 32 * (GX::LR + GH::LR); i += 256) fsm[i] = 0.f;

  // ---- weight fragments (B operand of 16x16x4: lane l holds B[k = 4 ks + (l >> 4)][col l & 15]) ----
  constexpr float GSC = ACT == ACT_TANH ? -2.f * kLog2e : ACT == ACT_SIGMOID ? -kLog2e : 1.f;
  const float sc = TAN ? 1.f : (q == 2 ? GSC : -kLog2e);
  float uf[GH::KS][FNT];
  float wf[NWR][FNT];
  float bq[FNT];
#pragma unroll
  for (int n = 0; n < FNT; ++n) {
    const int u = ub + 4 * n;
    const bool ok = u < FH;
    const int cl = q * FH + (ok ? u : FH - 1);
#pragma unroll
    for (int ks = 0; ks < GH::KS; ++ks) {
      const float v = U[(4 * ks + g) * FG + cl];  // k = 4 ks + g < 100 always
      uf[ks][n] = ok ? v * sc : 0.f;
      // U^T lives in the accumulator half of the register file (MFMA B operands may be AGPRs):
      // the VGPR half stays free for W^T, the loads in flight and the gate math
      asm volatile("" : "+a"(uf[ks][n]));
    }
#pragma unroll
    for (int ks = 0; ks < GX::KS; ++ks) {
      const int k = 4 * ks + g;
      const float v = W[min(k, KX - 1) * FG + cl];
      const float wv = (ok && k < KX) ? v * sc : 0.f;
      if (ks < NWR) {
        wf[ks < NWR ? ks : 0][n] = wv;
        if (ks >= 8) asm volatile("" : "+a"(wf[ks < NWR ? ks : 0][n]));  // (K = 100: 4 of its 12 k-steps)
      }
      else wl[(((ks - NWR) * 4 + w) * FNT + n) * 64 + lane] = wv;
    }
    const float bv = bias ? bias[cl] : 0.f;
    bq[n] = (!TAN && ok) ? bv * sc : 0.f;
  }
  // per-lane gate nonlinearity y = lin ? s : am * rcp(1 + exp2(s)) + bm (pre-scaled s)
  const bool glin = !TAN && ACT == ACT_LINEAR && q == 2;
  const float am = (ACT == ACT_TANH && q == 2) ? 2.f : 1.f, bm = (ACT == ACT_TANH && q == 2) ? -1.f : 0.f;
  // LDS element offsets: A-fragment reads (row l & 15, k-group g) and the h write of (row 4 g + q, unit ub + 4 n)
  const int ax = (lane & 15) * GX::LR + g * GX::KQ, ah = (lane & 15) * GH::LR + g * GH::KQ;
  const int hw = (4 * g + q) * GH::LR + j4 * GH::KQ + 7 * w;

  for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
    const int row0 = rb * 32;
    const rsrc_t rx = ftile_rsrc(x, row0, B, Tn, KX);
    const rsrc_t rh = ftile_rsrc(hs, row0, B, Tn, FH);
    const rsrc_t rt = ftape_rsrc(TAPE ? tape : nullptr, rb, nrb, Tn);  // primal (or tangent) tape out
    const rsrc_t rp = ftape_rsrc(TAN ? ptape : nullptr, rb, nrb, Tn);  // tangent: the primal tape
    // byte offsets at step 0 of this lane's (row 16 m + 4 g + q, unit ub) in (B,T,H) (the descriptor
    // covers rows < B only, so a row past B is out of range by itself); every offset below is
    // (base + t * step stride) + an immediate, so nothing per tile is hoisted out of the step loop
    int vp1[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) vp1[m] = ((16 * m + 4 * g + q) * Tn * FH + ub) * 4;
    const int tl = ftape_lane(w, lane), tcl = ftape_cell(w, lane);
    float cprev[TAN ? 2 : 1][FNT];  // tangent: c_{t-1} of the primal (carried)
    if constexpr (TAN) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < FNT; ++n) cprev[m][n] = 0.f;
    }
    float cst[2][FNT];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < FNT; ++n) cst[m][n] = 0.f;
    FXPart<KX> xp;
    xp.set(Tn, tid);
    xp.load(rx, Tn, 0, true);
    for (int i = tid; i < 32 * GH::LR; i += 256) hb[i] = 0.f;  // h_{-1} = 0
    xp.to_lds(xb, trash);
    __syncthreads();
    for (int t = 0; t < Tn; ++t) {
      const float* xcur = xb + (t & 1) * 32 * GX::LR;
      const float* hcur = hb + (t & 1) * 32 * GH::LR;
      float* hnext = hb + ((t + 1) & 1) * 32 * GH::LR;
      xp.load(rx, Tn, t + 1, t + 1 < Tn);  // x_{t+1}: lands during this step's MFMAs
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        // tangent: the primal gates and c_t of this lane's (row, unit), from its own tape slots;
        // issued before this half's MFMAs, consumed after them
        f32x4 pg[TAN ? FNT : 1];
        float pc[TAN ? FNT : 1];
        const int p1 = vp1[m] + t * FH * 4, tb = t * FT_STEP * 4;
        if constexpr (TAN) {
#pragma unroll
          for (int n = 0; n < FNT; ++n) {
            const bool tok = !(w == 3 && n >= 4);
            pg[n] = ld4(rp, tok ? tl + tb + ftape_slot(m, n) : kOOB);
            pc[n] = ld1(rp, tok ? tcl + tb + ftape_slot(m, n) : kOOB, 0);
          }
        }
        f32x4 acc[FNT];
#pragma unroll
        for (int n = 0; n < FNT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};  // (inline-constant C; bias added below)
        // ---- z = x_t W (+ b) ----
#pragma unroll
        for (int j = 0; j < GX::NJ; ++j) {
          const f32x4 a4 = *reinterpret_cast<const f32x4*>(xcur + ax + 16 * m * GX::LR + 4 * j);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int ks = 4 * j + s;
            if (ks >= GX::KS) break;
#pragma unroll
            for (int n = 0; n < FNT; ++n) {
              const float bw = ks < NWR ? wf[ks < NWR ? ks : 0][n] : wl[(((ks - NWR) * 4 + w) * FNT + n) * 64 + lane];
              acc[n] = mma4(a4[s], bw, acc[n]);
            }
          }
          __builtin_amdgcn_sched_barrier(0);  // bound the live range of hoisted fragment reads
        }
        // ---- + h_{t-1} U ----
#pragma unroll
        for (int j = 0; j < GH::NJ; ++j) {
          const f32x4 a4 = *reinterpret_cast<const f32x4*>(hcur + ah + 16 * m * GH::LR + 4 * j);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int ks = 4 * j + s;
            if (ks >= GH::KS) break;
#pragma unroll
            for (int n = 0; n < FNT; ++n) acc[n] = mma4(a4[s], uf[ks][n], acc[n]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        // ---- gate math, cell update, stores (row 16 m + 4 g + q, unit ub + 4 n after the transpose) ----
#pragma unroll
        for (int n = 0; n < FNT; ++n) {
          const bool tok = !(w == 3 && n >= 4);  // wave 3's tiles 4..6 are padding units 100..111
          const int v1 = tok ? p1 + 16 * n : kOOB;
          float hv;
          if constexpr (!TAN) {
            float y[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float s = acc[n][i] + bq[n];
              const float e = am * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(s)) + bm;
              y[i] = glin ? s : e;
            }
            quad_transpose(y, q);  // y = (i, f, g, o) of (row, unit)
            const float cn = y[1] * cst[m][n] + y[0] * y[2];
            float ca;
            if constexpr (ACT == ACT_TANH) ca = 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(GSC * cn)) - 1.f;
            else if constexpr (ACT == ACT_SIGMOID) ca = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(GSC * cn));
            else ca = cn;
            hv = tok ? y[3] * ca : 0.f;
            cst[m][n] = cn;
            if constexpr (TAPE) {
              st4(f32x4{y[0], y[1], y[2], y[3]}, rt, tok ? tl + tb + ftape_slot(m, n) : kOOB);
              st1(cn, rt, tok ? tcl + tb + ftape_slot(m, n) : kOOB, 0);
            }
          } else {
            // zdot of (row, unit) for all four gates: transpose the accumulator quad
            float zd[4] = {acc[n][0], acc[n][1], acc[n][2], acc[n][3]};
            quad_transpose(zd, q);
            const f32x4 y = pg[n];
            const float idot = y[0] * (1.f - y[0]) * zd[0], fdot = y[1] * (1.f - y[1]) * zd[1];
            const float gdot = act_dy(ACT, y[2]) * zd[2], odot = y[3] * (1.f - y[3]) * zd[3];
            const float c = pc[n];
            float cdn = fdot * cprev[m][n] + y[1] * cst[m][n] + idot * y[2] + y[0] * gdot;
            const float ca = act_f(ACT, c);
            float hd = odot * ca + y[3] * act_dy(ACT, ca) * cdn;
            if (!tok) { cdn = 0.f; hd = 0.f; }
            cst[m][n] = cdn;
            cprev[m][n] = c;
            hv = hd;
            st4(f32x4{zd[0], zd[1], zd[2], zd[3]}, rt, tok ? tl + tb + ftape_slot(m, n) : kOOB);
            st1(cdn, rt, tok ? tcl + tb + ftape_slot(m, n) : kOOB, 0);
          }
          hnext[hw + 16 * m * GH::LR + n] = hv;  // padded units (u < 112) write their zeros
          st1(hv, rh, v1, 0);
        }
      }
      xp.to_lds(xb + ((t + 1) & 1) * 32 * GX::LR, trash);
      lds_barrier();
    }
  }
}

// ==========================================================================================
// BPTT (fp32): dZ_t = dL/dz_t (ops/reference.py lstm_seq_bwd) from the row-major fp32 tapes
// ==========================================================================================
// Same wave / lane decomposition as the forward: after the quad transpose lane (g, j4, q) of wave
// w owns (row 16 m + 4 g + q, unit 28 w + 4 n + j4) for m < 2, n < 7, and keeps that cell's dc.
// Per step, two phases between LDS barriers:
//   A. dh_rec = dz_{t+1} U^T on 16x16x4 MFMAs: A = the dz tile in LDS (k = 4 u' + q, row layout
//      [q][u'] so one ds_read_b128 feeds four k-steps), B = U^T fragments pinned in AGPRs; wave w
//      owns output column tiles 2 w, 2 w + 1 (16 units each) for both row halves (400 MFMAs), and
//      the step's tape / dH loads are issued before it so their latency hides under the MFMAs;
//   B. the cell adjoint math per (row, unit), dZ_t to HBM (row-major, for the weight gradient and the
//      input-gradient GEMM) and to the dz tile for the next step.
constexpr int BZ_KQ = 100, BZ_LR = 408, BH_LR = 116;  // dz tile: conflict-free b128 reads (scripted search)

// dZ_{t+1} leaves through 16-byte row-major stores read back from the dz tile during phase A of step
// t (the tile holds it anyway), and step t-1's tape loads are issued at the end of phase B of step t,
// reusing the registers just consumed: every load is older than the stores it could queue behind
// (vmcnt retires loads and stores in issue order), and every store is coalesced.
// step t's tape for the BPTT: the gate quad at t and c_{t-1} (c_t is carried from the step above)
__device__ __forceinline__ void bwdf_tape_load(f32x4& tg, float& tcp, float& tdh, rsrc_t rt, rsrc_t rdh, int og, int ocp,
                                               int p1, bool tok, bool prev) {
  tg = ld4(rt, tok ? og : kOOB);
  tcp = ld1(rt, (tok && prev) ? ocp : kOOB, 0);
  tdh = ld1(rdh, tok ? p1 : kOOB, 0);
}
// the same loads with the per-lane part of each offset in voffset (tl / tcl / vp) and the uniform part
// (step and slot) in soffset: no per-cell offset arithmetic on the VALU (the split BPTT is VALU-bound,
// profiles/r03_end/pmc_fp32.txt).  Out-of-range lanes: voffset kOOB (the range check is on voffset)
// HEAD: dH is the critic head's outer-product adjoint dH[b, t, u] = hdm * w[t, u] (hdm = the lane row's
// d[b], w = the head weight, (Tn, H) like one row of dH: same soffset, voffset hvo = the unit's
// offset), generated here instead of read from a materialised (B, Tn, H) tensor
template <bool HEAD>
__device__ __forceinline__ void bwdf_tape_load_u(f32x4& tg, float& tcp, float& tdh, rsrc_t rt, rsrc_t rdh, int tl, int tcl,
                                                 int vp, int sg, int sc, int sd, bool tok, bool prev, float hdm,
                                                 rsrc_t rhw, int hvo) {
  tg = ld4s(rt, tok ? tl : kOOB, sg);
  tcp = ld1(rt, (tok && prev) ? tcl : kOOB, sc);
  // (the product may contract into the consumer's add: one rounding fewer than a materialised dH, i.e.
  // within an ulp of it; an empty-asm barrier against that breaks the step schedule, +40 % per call)
  if constexpr (HEAD) tdh = hdm * ld1(rhw, tok ? hvo : kOOB, sd);
  else tdh = ld1(rdh, tok ? vp : kOOB, sd);
}
// the dz tile (32 rows x [q][u'], u' < 100) -> dZ[:, t, :] (row-major, 4H per row) in 16-byte chunks:
// threads 0..199 own chunk (tid % 100) of rows 2 k + tid / 100 (k < 16); the row step lives in the
// uniform soffset, so a thread holds one LDS and one global base (rows past B: voffset out of range)
struct BwdfStore {
  int lo, go, rr;
  __device__ __forceinline__ void set(int tid, int Tn) {
    rr = tid / 100;
    const int ch = tid - 100 * rr, qq = ch / 25, c = ch - 25 * qq;
    lo = (rr & 1) * BZ_LR + qq * BZ_KQ + 4 * c;
    go = tid < 200 ? (rr * Tn * FG + qq * FH + 4 * c) * 4 : kOOB;
  }
  __device__ __forceinline__ void store(const float* zt, rsrc_t rz, int Tn, int t, int nr) const {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(zt + lo + 2 * k * BZ_LR);
      st16(v, rz, 2 * k + rr < nr, go, (2 * k * Tn + t) * FG * 4);
    }
  }
};

// 16-row variant for the tangent reverse: threads 0..199 own chunk tid % 100 of rows 2 k + tid / 100
__device__ __forceinline__ void bwdf_store16(const float* zt, rsrc_t rz, int Tn, int t, int nr, int tid) {
  const int rr = tid / 100, ch = tid - 100 * rr, qq = ch / 25, c = ch - 25 * qq;
  const int lo = (rr & 1) * BZ_LR + qq * BZ_KQ + 4 * c;
  const int go = tid < 200 ? (rr * Tn * FG + qq * FH + 4 * c) * 4 : kOOB;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(zt + lo + 2 * k * BZ_LR);
    st16(v, rz, 2 * k + rr < nr, go, (2 * k * Tn + t) * FG * 4);
  }
}

// ------------------------------------------------------------------------------------------
// BPTT with a role split and a row-half pipeline (8 waves, two per SIMD).
//
// A BPTT that runs the step's MFMA phase (dh_rec = dz_{t+1} U^T) and its VALU phase (the cell
// adjoints) back to back in the same four waves leaves the matrix pipe idle through every VALU phase:
// 400 MFMAs = 12.8 k cycles of pipe time per wave and step against ~24 k measured.  A single wave
// cannot overlap them (in-order issue; the scheduler keeps the cell math in clumps between MFMA
// runs), so here the roles go to different waves that share a SIMD:
//   * waves 0..3 (MFMA role): U^T fragments in AGPRs (the same 2 column tiles per wave as before)
//     and nothing else; A(m, t) = rows m of dh_rec(t) -> the dh tile;
//   * waves 4..7 (cell role): the cell state, tape loads and dZ stores of units 28 w' .. 28 w' + 27;
//     B(m, t) = the cell adjoints of rows m, which overwrite rows m of the dz tile with dz_t.
// The two 16-row halves of a tile are independent recurrences (the A operand of row r is
// dz_{t+1}[r]), so one role works on one half while the other role works on the other half:
//   P1(t): B(0, t) || A(1, t)      P2(t): B(1, t) || A(0, t - 1)
// with one barrier after each.  The hardware interleaves the two waves of a SIMD, so the cell math
// issues while the matrix pipe runs.  Register budget: the MFMA role ~230 (200 AGPRs of U^T), the
// cell role ~150, two waves per SIMD.  dZ rows of a half leave during the half-phase after the one
// that completed them (the tile rows are stable for exactly that phase).  The dz / dh tiles start at
// zero (dz_T = 0, dh_rec(T - 1) = 0), so the first P1 and the last P2 need no special case
// (A(0, -1) is computed into dh rows 0 and never read).
template <int ACT>
__global__ void __launch_bounds__(512, 1)
lstmf_bwdp_kernel(const float* __restrict__ dH, const float* __restrict__ tape, const float* __restrict__ U,
                  float* __restrict__ dZ, int B, int Tn) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  float* zt = fsm;                  // dz tile [32][BZ_LR]: [q][u'] per row
  float* ht = zt + 32 * BZ_LR;      // dh_rec tile [32][BH_LR]
  float* trash = ht + 32 * BH_LR;   // [4 * BZ_KQ] written by padding cells, never read
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = wv & 3;             // wave index within the role
  const int q = lane & 3, g = lane >> 4, j4 = (lane & 15) >> 2, c16 = lane & 15;
  const int nrb = (B + 31) / 32;
  if (wv < 4) {
    // ---------------- MFMA role ----------------
    float ut[2][FH];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = 16 * (2 * w + e) + c16;
      const bool ok = j < FH;
#pragma unroll
      for (int k = 0; k < FH; ++k) {
        const float v = U[(ok ? j : 0) * FG + g * FH + k];
        ut[e][k] = ok ? v : 0.f;  // (arch VGPRs: at two waves per SIMD the role fits in 256)
      }
    }
    // rows of half M of dh_rec = dz[rows M] U^T -> the dh tile
    auto half_a = [&](auto MA_) {
      constexpr int M = decltype(MA_)::value;
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      const float* ar = zt + (16 * M + c16) * BZ_LR + g * BZ_KQ;
#pragma unroll
      for (int jj = 0; jj < FH / 4; ++jj) {
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(ar + 4 * jj);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc[0] = mma4(a4[s], ut[0][4 * jj + s], acc[0]);
          acc[1] = mma4(a4[s], ut[1][4 * jj + s], acc[1]);
        }
        if ((jj & 3) == 3) __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int col = 16 * (2 * w + e) + c16;
        if (2 * w + e < 7) {  // (wave 3's second tile is past the 112-unit tile: uniform skip)
#pragma unroll
          for (int i = 0; i < 4; ++i) ht[(16 * M + 4 * g + i) * BH_LR + col] = acc[e][i];
        }
      }
    };
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      for (int i = tid; i < 32 * BZ_LR; i += 512) zt[i] = 0.f;  // dz_T = 0
      for (int i = tid; i < 32 * BH_LR; i += 512) ht[i] = 0.f;  // dh_rec(T - 1) = 0
      __syncthreads();
      for (int t = Tn - 1; t >= 0; --t) {
        half_a(std::integral_constant<int, 1>{});  // P1(t): A(1, t)
        lds_barrier();
        half_a(std::integral_constant<int, 0>{});  // P2(t): A(0, t - 1)
        lds_barrier();
      }
      __syncthreads();
    }
  } else {
    // ---------------- cell role ----------------
    const int ct = tid - 256;
    const int ub = FUW * w + j4;
    const int hr = (4 * g + q) * BH_LR + ub, zw = (4 * g + q) * BZ_LR + ub;
    // dZ store share: threads 0..199 of the role own chunk ct % 100 of rows 2 k + ct / 100 (k < 16)
    const int srr = ct / 100, sch = ct - 100 * srr, sqq = sch / 25, sc = sch - 25 * sqq;
    const int slo = (srr & 1) * BZ_LR + sqq * BZ_KQ + 4 * sc;
    const int sgo = ct < 200 ? (srr * Tn * FG + sqq * FH + 4 * sc) * 4 : kOOB;
    const int tl = ftape_lane(w, lane), tcl = ftape_cell(w, lane);
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      const int row0 = rb * 32;
      const rsrc_t rdh = ftile_rsrc(dH, row0, B, Tn, FH), rt = ftape_rsrc(tape, rb, nrb, Tn);
      const rsrc_t rz = ftile_rsrc(dZ, row0, B, Tn, FG);
      const int nr = min(32, B - row0);
      int vp1[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) vp1[m] = ((16 * m + 4 * g + q) * Tn * FH + ub) * 4;
      float dc[2][FNT], tc[2][FNT];
      f32x4 tg[2][FNT];
      float tcp[2][FNT], tdh[2][FNT];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < FNT; ++n) {
          const bool tok = !(w == 3 && n >= 4);
          const int T1 = Tn - 1;
          dc[m][n] = 0.f;
          tc[m][n] = ld1(rt, tok ? tcl + T1 * FT_STEP * 4 + ftape_slot(m, n) : kOOB, 0);  // c_{T-1}
          bwdf_tape_load(tg[m][n], tcp[m][n], tdh[m][n], rt, rdh, tl + T1 * FT_STEP * 4 + ftape_slot(m, n),
                         tcl + (T1 - 1) * FT_STEP * 4 + ftape_slot(m, n), vp1[m] + T1 * FH * 4 + 16 * n, tok, T1 > 0);
        }
      for (int i = tid; i < 32 * BZ_LR; i += 512) zt[i] = 0.f;
      for (int i = tid; i < 32 * BH_LR; i += 512) ht[i] = 0.f;
      __syncthreads();
      // rows of half M of the dz tile (dz at step ts) -> dZ[:, ts, :]
      auto store_half = [&](auto M_, int ts) {
        constexpr int M = decltype(M_)::value;
#pragma unroll
        for (int k = 8 * M; k < 8 * M + 8; ++k) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(zt + slo + 2 * k * BZ_LR);
          st16(v, rz, 2 * k + srr < nr, sgo, (2 * k * Tn + ts) * FG * 4);
        }
      };
      // cell adjoints of row half M at step t; each cell then issues step t - 1's tape loads
      auto half_b = [&](auto M_, int t) {
        constexpr int m = decltype(M_)::value;
#pragma unroll
        for (int n = 0; n < FNT; ++n) {
          const bool tok = !(w == 3 && n >= 4);
          const float ig = tg[m][n][0], fg = tg[m][n][1], gg = tg[m][n][2], og = tg[m][n][3];
          const float dht = tdh[m][n] + ht[hr + 16 * m * BH_LR + 4 * n];
          const float ca = act_f(ACT, tc[m][n]);
          const float dov = dht * ca;
          const float dct = dc[m][n] + dht * og * act_dy(ACT, ca);
          dc[m][n] = tok ? dct * fg : 0.f;
          float z4[4];
          z4[0] = dct * gg * ig * (1.f - ig);
          z4[1] = dct * tcp[m][n] * fg * (1.f - fg);
          z4[2] = dct * ig * act_dy(ACT, gg);
          z4[3] = dov * og * (1.f - og);
          float* zd = tok ? zt + zw + 16 * m * BZ_LR + 4 * n : trash;  // padding cells: trash row
#pragma unroll
          for (int k = 0; k < 4; ++k) zd[k * BZ_KQ] = z4[k];
          tc[m][n] = tcp[m][n];  // c_{t-1} is the next step's c
          const int tp = t > 0 ? t - 1 : 0;
          bwdf_tape_load(tg[m][n], tcp[m][n], tdh[m][n], rt, rdh, tl + tp * FT_STEP * 4 + ftape_slot(m, n),
                         tcl + (tp - 1) * FT_STEP * 4 + ftape_slot(m, n), vp1[m] + tp * FH * 4 + 16 * n,
                         tok && t > 0, tp > 0);
        }
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      for (int t = Tn - 1; t >= 0; --t) {
        if (t < Tn - 1) store_half(I1{}, t + 1);  // rows 16..31 of dz_{t+1}: stable until P2(t)
        half_b(I0{}, t);                          // P1(t): B(0, t)
        lds_barrier();
        store_half(I0{}, t);                      // rows 0..15 of dz_t: stable until P1(t - 1)
        half_b(I1{}, t);                          // P2(t): B(1, t)
        lds_barrier();
      }
      store_half(I1{}, 0);
      __syncthreads();  // (the tiles are re-zeroed for the next row block)
    }
  }
}

// ==========================================================================================
// tangent reverse (fp32): (dZ, dZdot) of the reverse-over-tangent pass (ops/reference.py
// lstm_seq_tbwd) from the primal and tangent tapes of lstmf_fwd<TAPE> / lstmf_fwd<TAN>
// ==========================================================================================
// ------------------------------------------------------------------------------------------
// tangent reverse with the role split of lstmf_bwdp_kernel: 32-row tiles whose 16-row halves are
// pipelined (P1(t): cells of rows 0-15 || MFMAs of rows 16-31; P2(t): cells of rows 16-31 ||
// MFMAs of rows 0-15 of the previous step), MFMA waves 0..3 (U^T in VGPRs, both adjoint streams:
// 400 MFMAs per half-phase) and cell waves 4..7.  The cell waves carry 4 values per cell for both
// halves (c, cdot and the two adjoint carries) and ONE set of step loads (gates, zdot, c_{t-1},
// cdot_{t-1}, dH, dHd: 12 per cell): the set for the other half is issued right after a half's
// cells, and lands while the MFMA waves finish the half-phase.
#ifndef HFREP_TBWD_CELLGROUP
#define HFREP_TBWD_CELLGROUP 2
#endif
template <int ACT, bool HEAD = false>
__global__ void __launch_bounds__(512, 1)
lstmf_tbwdp_kernel(const float* __restrict__ dH, const float* __restrict__ dHd, const float* __restrict__ tape,
                   const float* __restrict__ ttape, const float* __restrict__ U, float* __restrict__ dZ,
                   float* __restrict__ dZd, int B, int Tn, const float* __restrict__ hd, const float* __restrict__ hdd,
                   const float* __restrict__ hw) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  float* zt = fsm;                   // dz tile     [32][BZ_LR]
  float* zdt = zt + 32 * BZ_LR;      // dzdot tile  [32][BZ_LR]
  float* ht = zdt + 32 * BZ_LR;      // dz U^T      [32][BH_LR]
  float* hdt = ht + 32 * BH_LR;      // dzdot U^T   [32][BH_LR]
  float* trash = hdt + 32 * BH_LR;   // [4 * BZ_KQ] padding-cell writes
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = wv & 3;
  const int q = lane & 3, g = lane >> 4, j4 = (lane & 15) >> 2, c16 = lane & 15;
  const int nrb = (B + 31) / 32;
  if (wv < 4) {
    // ---------------- MFMA role ----------------
    float ut[2][FH];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = 16 * (2 * w + e) + c16;
      const bool ok = j < FH;
#pragma unroll
      for (int k = 0; k < FH; ++k) {
        const float v = U[(ok ? j : 0) * FG + g * FH + k];
        ut[e][k] = ok ? v : 0.f;
      }
    }
    // rows of half M of (dz, dzdot) U^T, one adjoint stream after the other (8 accumulator
    // registers live: U^T takes 200 of the role's 256 VGPRs)
    auto half_a = [&](auto MA_) {
      constexpr int M = decltype(MA_)::value;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        const float* ar = (st ? zdt : zt) + (16 * M + c16) * BZ_LR + g * BZ_KQ;
#pragma unroll
        for (int jj = 0; jj < FH / 4; ++jj) {
          const f32x4 a4 = *reinterpret_cast<const f32x4*>(ar + 4 * jj);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            acc[0] = mma4(a4[s], ut[0][4 * jj + s], acc[0]);
            acc[1] = mma4(a4[s], ut[1][4 * jj + s], acc[1]);
          }
          if ((jj & 1) == 1) __builtin_amdgcn_sched_barrier(0);
        }
        float* hd = st ? hdt : ht;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int col = 16 * (2 * w + e) + c16;
          if (2 * w + e < 7) {
#pragma unroll
            for (int i = 0; i < 4; ++i) hd[(16 * M + 4 * g + i) * BH_LR + col] = acc[e][i];
          }
        }
      }
    };
    // the dz / dzdot stores ride on the MFMA role (they were 6 % of the cell role's time, which
    // sets the half-phase length): threads 0..199 own chunk tid % 100 of rows 2 k + tid / 100; a
    // half's rows are stable for exactly the half-phase after the one that completed them
    const int srr = tid / 100, sch = tid - 100 * srr, sqq = sch / 25, sc = sch - 25 * sqq;
    const int slo = (srr & 1) * BZ_LR + sqq * BZ_KQ + 4 * sc;
    const int sgo = tid < 200 ? (srr * Tn * FG + sqq * FH + 4 * sc) * 4 : kOOB;
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      const int row0 = rb * 32;
      const rsrc_t rz = ftile_rsrc(dZ, row0, B, Tn, FG), rzd = ftile_rsrc(dZd, row0, B, Tn, FG);
      const int nr = min(32, B - row0);
      auto store_half = [&](auto M_, int ts) {
        constexpr int M = decltype(M_)::value;
#pragma unroll
        for (int k = 8 * M; k < 8 * M + 8; ++k) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(zt + slo + 2 * k * BZ_LR);
          const f32x4 vd = *reinterpret_cast<const f32x4*>(zdt + slo + 2 * k * BZ_LR);
          const bool ok = 2 * k + srr < nr;
          const int so = (2 * k * Tn + ts) * FG * 4;
          st16(v, rz, ok, sgo, so);
          st16(vd, rzd, ok, sgo, so);
          if (k & 1) __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      for (int i = tid; i < 2 * 32 * (BZ_LR + BH_LR); i += 512) zt[i] = 0.f;  // all four tiles
      __syncthreads();
      for (int t = Tn - 1; t >= 0; --t) {
        if (t < Tn - 1) store_half(I1{}, t + 1);  // rows 16..31 of dz_{t+1}: stable during P1(t)
        half_a(I1{});
        lds_barrier();
        store_half(I0{}, t);                      // rows 0..15 of dz_t: stable during P2(t)
        half_a(I0{});
        lds_barrier();
      }
      store_half(I1{}, 0);
      __syncthreads();
    }
  } else {
    // ---------------- cell role ----------------
    const int ct = tid - 256;
    const int ub = FUW * w + j4;
    const int hr = (4 * g + q) * BH_LR + ub, zw = (4 * g + q) * BZ_LR + ub;
    const int srr = ct / 100, sch = ct - 100 * srr, sqq = sch / 25, sc = sch - 25 * sqq;
    const int slo = (srr & 1) * BZ_LR + sqq * BZ_KQ + 4 * sc;
    const int sgo = ct < 200 ? (srr * Tn * FG + sqq * FH + 4 * sc) * 4 : kOOB;
    const int tl = ftape_lane(w, lane), tcl = ftape_cell(w, lane);
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      const int row0 = rb * 32;
      const rsrc_t rdh = ftile_rsrc(dH, row0, B, Tn, FH), rdhd = ftile_rsrc(dHd, row0, B, Tn, FH);
      const rsrc_t rt = ftape_rsrc(tape, rb, nrb, Tn), rtt = ftape_rsrc(ttape, rb, nrb, Tn);
      const rsrc_t rz = ftile_rsrc(dZ, row0, B, Tn, FG), rzd = ftile_rsrc(dZd, row0, B, Tn, FG);
      const int nr = min(32, B - row0);
      int vp1[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) vp1[m] = ((16 * m + 4 * g + q) * Tn * FH + ub) * 4;
      // HEAD: dH = hd (x) w, dHd = hdd (x) w generated per cell (a null factor: that adjoint is zero)
      float hdv[2] = {0.f, 0.f}, hddv[2] = {0.f, 0.f};
      const rsrc_t rhw = make_rsrc(hw, HEAD ? Tn * FH * 4 : 0);
      if constexpr (HEAD) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int r = row0 + 16 * m + 4 * g + q;
          hdv[m] = (hd && r < B) ? hd[r] : 0.f;
          hddv[m] = (hdd && r < B) ? hdd[r] : 0.f;
        }
      }
      const int hvo = ub * 4;
      float tc[2][FNT], tcd[2][FNT], acn[2][FNT], acdn[2][FNT];
      f32x4 tg[FNT], tz[FNT];
      float tcp[FNT], tcdp[FNT], tdh[FNT], tdhd[FNT];
      // the step loads of half M at step tt (one register set, reused by the two halves in turn).
      // The per-lane part of every address is one of four VGPRs (tl, tcl, vp1[m]); the cell's slot
      // and the step go into the uniform soffset, so no per-cell offset registers are hoisted
      // (out-of-range lanes: voffset kOOB, which the range check drops whatever the soffset)
      auto load_half = [&](auto M_, int tt, bool on) {
        constexpr int m = decltype(M_)::value;
        const int tp = tt > 0 ? tt - 1 : 0;
#pragma unroll
        for (int n = 0; n < FNT; ++n) {
          const bool tok = on && !(w == 3 && n >= 4);
          const int sg = tt * FT_STEP * 4 + ftape_slot(m, n), sc = tp * FT_STEP * 4 + ftape_slot(m, n);
          const int sd = tt * FH * 4 + 16 * n;
          tg[n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rt, tok ? tl : kOOB, sg, 0));
          tz[n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtt, tok ? tl : kOOB, sg, 0));
          tcp[n] = ld1(rt, (tok && tt > 0) ? tcl : kOOB, sc);
          tcdp[n] = ld1(rtt, (tok && tt > 0) ? tcl : kOOB, sc);
          if constexpr (HEAD) {
            const float wv = ld1(rhw, tok ? hvo : kOOB, sd);
            tdh[n] = hdv[m] * wv;
            tdhd[n] = hddv[m] * wv;
          } else {
            tdh[n] = ld1(rdh, tok ? vp1[m] : kOOB, sd);
            tdhd[n] = ld1(rdhd, tok ? vp1[m] : kOOB, sd);
          }
        }
      };
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < FNT; ++n) {
          const bool tok = !(w == 3 && n >= 4);
          const int oc = tcl + (Tn - 1) * FT_STEP * 4 + ftape_slot(m, n);
          acn[m][n] = 0.f;
          acdn[m][n] = 0.f;
          tc[m][n] = ld1(rt, tok ? oc : kOOB, 0);
          tcd[m][n] = ld1(rtt, tok ? oc : kOOB, 0);
        }
      load_half(std::integral_constant<int, 0>{}, Tn - 1, true);
      for (int i = tid; i < 2 * 32 * (BZ_LR + BH_LR); i += 512) zt[i] = 0.f;
      __syncthreads();
      auto half_b = [&](auto M_) {
        constexpr int m = decltype(M_)::value;
#pragma unroll
        for (int n = 0; n < FNT; ++n) {
          const bool tok = !(w == 3 && n >= 4);
          const float i_ = tg[n][0], f_ = tg[n][1], g_ = tg[n][2], o_ = tg[n][3];
          const float zdi = tz[n][0], zdf = tz[n][1], zdg = tz[n][2], zdo = tz[n][3];
          const float c = tc[m][n], cd = tcd[m][n], cp = tcp[n], cdp = tcdp[n];
          const float si = i_ * (1.f - i_), sf = f_ * (1.f - f_), so = o_ * (1.f - o_), sg = act_dy(ACT, g_);
          const float idot = si * zdi, fdot = sf * zdf, gdot = sg * zdg, odot = so * zdo;
          const float ca = act_f(ACT, c), d1 = act_dy(ACT, ca), d2 = act_d2y(ACT, ca);
          const int hi = hr + 16 * m * BH_LR + 4 * n;
          const float a_h = tdh[n] + ht[hi], a_hd = tdhd[n] + hdt[hi];
          const float a_od = a_hd * ca;
          const float a_o = a_h * ca + a_hd * d1 * cd;
          const float a_cd = acdn[m][n] + a_hd * o_ * d1;
          const float a_c = acn[m][n] + a_h * o_ * d1 + a_hd * (odot * d1 + o_ * d2 * cd);
          const float a_fd = a_cd * cp, a_id = a_cd * g_, a_gd = a_cd * i_;
          const float a_f = a_c * cp + a_cd * cdp;
          const float a_i = a_c * g_ + a_cd * gdot;
          const float a_g = a_c * i_ + a_cd * idot;
          acn[m][n] = tok ? a_c * f_ + a_cd * fdot : 0.f;
          acdn[m][n] = tok ? a_cd * f_ : 0.f;
          const float s2i = si * (1.f - 2.f * i_), s2f = sf * (1.f - 2.f * f_), s2o = so * (1.f - 2.f * o_);
          const float s2g = act_d2y(ACT, g_);
          float zd4[4], z4[4];
          zd4[0] = a_id * si; zd4[1] = a_fd * sf; zd4[2] = a_gd * sg; zd4[3] = a_od * so;
          z4[0] = a_i * si + a_id * s2i * zdi;
          z4[1] = a_f * sf + a_fd * s2f * zdf;
          z4[2] = a_g * sg + a_gd * s2g * zdg;
          z4[3] = a_o * so + a_od * s2o * zdo;
          const int zo = zw + 16 * m * BZ_LR + 4 * n;
          float* zp = tok ? zt + zo : trash;
          float* zdp = tok ? zdt + zo : trash;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            zp[k * BZ_KQ] = z4[k];
            zdp[k * BZ_KQ] = zd4[k];
          }
          tc[m][n] = cp;
          tcd[m][n] = cdp;
          // HFREP_TBWD_CELLGROUP cells' temporaries per schedule region: 2 (13.80 -> 13.45 ms per call at
          // B = 262 144; one cell at a time was the round-4 schedule, seven 13.56 ms:
          // profiles/r05_tbwd/README.md)
          if ((n + 1) % HFREP_TBWD_CELLGROUP == 0 || n == FNT - 1) __builtin_amdgcn_sched_barrier(0);
        }
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      for (int t = Tn - 1; t >= 0; --t) {
        half_b(I0{});                             // P1(t): B(0, t)
        __builtin_amdgcn_sched_barrier(0);        //   (the load set is free only after the cells)
        load_half(I1{}, t, true);                 //   then half 1's loads for P2(t)
        lds_barrier();
        half_b(I1{});                             // P2(t): B(1, t)
        __builtin_amdgcn_sched_barrier(0);
        load_half(I0{}, t > 0 ? t - 1 : 0, t > 0);  //   then half 0's loads for P1(t - 1)
        lds_barrier();
      }
      __syncthreads();
    }
  }
}

// ==========================================================================================
// fused fp32 LSTM weight gradients
// ==========================================================================================
// slab[z] ((K + H + 1) x 4H) = sum over workgroup z's rows m of [x_m | h_{m-1} | 1]^T dz_m, plus the
// tangent segment [xd_m | hd_{m-1} | 0]^T dzd_m when given; one fixed-order reduce folds the slabs
// into gW / gU / gb (launch_lstm_wgrad2_reduce).  The v1 fp32 path ran one tiled GEMM per product
// (X^T dZ, H^T dZ, Xd^T dZd, Hd^T dZd: each re-reading dZ, ~35 TF/s, profiles/r02_fp32): here every
// (row chunk) is staged once and feeds all products.
//
// 8 waves (2 per SIMD), 16-row chunks = four 16x16x4 k-steps; output tiles 16 x 16: wave w owns the
// full i range of column tiles 3 w .. 3 w + 2 plus i-tiles 2 w, 2 w + 1 of the 25th column tile,
// i.e. 3 NI + 2 accumulators (K = 100: 41 x 4 AGPRs), the same MFMA count on every wave.
// Chunks are double-buffered in LDS through a register prefetch of the next chunk.
constexpr int WF_R = 16, WF_LA = 272, WF_LD = 400;  // row strides = 16 mod 64 dwords: conflict-free b32 reads
template <int KX>
struct WFGeo {
  static constexpr int KR = KX + FH + 1;
  static constexpr int NI = (KR + 15) / 16;
  static_assert(NI <= 16 && 16 * 16 <= WF_LA, "wgrad i tiles");
  static constexpr int NX4 = WF_R * KX / 4, NH4 = WF_R * FH / 4, ND4 = WF_R * FG / 4;
  static constexpr int JX = (NX4 + 511) / 512, JH = (NH4 + 511) / 512, JD = (ND4 + 511) / 512;
};

template <int KX, int XR = KX>  // XR: X row stride in floats (35: a 36-column image, column 35 zero)
__global__ void __launch_bounds__(512)
lstmf_wgrad_kernel(const float* __restrict__ X, const float* __restrict__ Hs, const float* __restrict__ D,
                   const float* __restrict__ Xd, const float* __restrict__ Hds, const float* __restrict__ Dd,
                   float* __restrict__ slab, int M, int Tn, int rows_per_wg) {
  using WG = WFGeo<KX>;
  constexpr int NI = WG::NI, KR = WG::KR;
  __shared__ __attribute__((aligned(16))) float As[2][WF_R * WF_LA];
  __shared__ __attribute__((aligned(16))) float Ds[2][WF_R * WF_LD];
  __shared__ __attribute__((aligned(16))) float trash4[4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int mb = blockIdx.x * rows_per_wg, me = min(M, mb + rows_per_wg);
  for (int i = tid; i < 2 * WF_R * WF_LA; i += 512) (&As[0][0])[i] = 0.f;

  f32x4 acc[NI][3], accx[2];
#pragma unroll
  for (int it = 0; it < NI; ++it)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) acc[it][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  accx[0] = accx[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ie0 = min(2 * w, 15), ie1 = min(2 * w + 1, 15);  // i tiles >= NI read LDS zeros

  // per-thread chunk loads: X (JX), H_{m-1} (JH), D (JD) float4s
  f32x4 vx[WG::JX], vh[WG::JH], vd[WG::JD];
  for (int seg = 0; seg < (Xd ? 2 : 1); ++seg) {
    const float* Xs = seg ? Xd : X;
    const float* Hq = seg ? Hds : Hs;
    const float* Dq = seg ? Dd : D;
    // descriptors based at this workgroup's first row (row mb - 1 for the shifted H): the byte
    // offsets stay 32-bit however large M is (a whole-tensor base overflowed past 1.34 M rows of dZ)
    const int hb = mb > 0 ? mb - 1 : 0, nr = me > mb ? me - mb : 0;
    const rsrc_t rx = make_rsrc(Xs + (size_t)mb * XR, nr * XR * 4);
    const rsrc_t rh = make_rsrc(Hq + (size_t)hb * FH, (nr ? me - hb : 0) * FH * 4);
    const rsrc_t rd = make_rsrc(Dq + (size_t)mb * FG, nr * FG * 4);
    auto load = [&](int m0) {
#pragma unroll
      for (int j = 0; j < WG::JX; ++j) {
        const int e = tid + 512 * j, r = e / (KX / 4), c = e - r * (KX / 4);
        const bool ok = e < WG::NX4 && m0 + r < me;
        vx[j] = ldx4<XR>(rx, ok ? ((m0 - mb + r) * XR + 4 * c) * 4 : kOOB, 0, 4 * c);
      }
#pragma unroll
      for (int j = 0; j < WG::JH; ++j) {
        const int e = tid + 512 * j, r = e / (FH / 4), c = e - r * (FH / 4);
        const int m = m0 + r;
        const bool ok = e < WG::NH4 && m < me && (m % Tn) != 0;  // h_{-1} = 0 at t = 0
        vh[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, ok ? ((m - 1 - hb) * FH + 4 * c) * 4 : kOOB, 0, 0));
      }
#pragma unroll
      for (int j = 0; j < WG::JD; ++j) {
        const int e = tid + 512 * j, r = e / (FG / 4), c = e - r * (FG / 4);
        const bool ok = e < WG::ND4 && m0 + r < me;
        vd[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, ok ? ((m0 - mb + r) * FG + 4 * c) * 4 : kOOB, 0, 0));
      }
    };
    auto to_lds = [&](int buf) {
#pragma unroll
      for (int j = 0; j < WG::JX; ++j) {
        const int e = tid + 512 * j, r = e / (KX / 4), c = e - r * (KX / 4);
        *reinterpret_cast<f32x4*>(e < WG::NX4 ? &As[buf][r * WF_LA + 4 * c] : trash4) = vx[j];
      }
#pragma unroll
      for (int j = 0; j < WG::JH; ++j) {
        const int e = tid + 512 * j, r = e / (FH / 4), c = e - r * (FH / 4);
        *reinterpret_cast<f32x4*>(e < WG::NH4 ? &As[buf][r * WF_LA + KX + 4 * c] : trash4) = vh[j];
      }
#pragma unroll
      for (int j = 0; j < WG::JD; ++j) {
        const int e = tid + 512 * j, r = e / (FG / 4), c = e - r * (FG / 4);
        *reinterpret_cast<f32x4*>(e < WG::ND4 ? &Ds[buf][r * WF_LD + 4 * c] : trash4) = vd[j];
      }
    };
    __syncthreads();  // (previous segment's reads done)
    if (tid < 2 * WF_R) As[tid >> 4][(tid & 15) * WF_LA + KR - 1] = seg ? 0.f : 1.f;  // the bias column
    if (mb < me) {
      load(mb);
      to_lds(0);
    }
    __syncthreads();
    int buf = 0;
    for (int m0 = mb; m0 < me; m0 += WF_R) {
      const bool more = m0 + WF_R < me;
      if (more) load(m0 + WF_R);
      const float* A_ = As[buf];
      const float* D_ = Ds[buf];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const float* ar = A_ + (4 * ks + g) * WF_LA + c16;
        const float* dr = D_ + (4 * ks + g) * WF_LD + c16;
        float a[NI], b[3];
#pragma unroll
        for (int it = 0; it < NI; ++it) a[it] = ar[16 * it];
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) b[jj] = dr[16 * (3 * w + jj)];
        const float bx = dr[16 * 24], ax0 = ar[16 * ie0], ax1 = ar[16 * ie1];
#pragma unroll
        for (int it = 0; it < NI; ++it)
#pragma unroll
          for (int jj = 0; jj < 3; ++jj) acc[it][jj] = mma4(a[it], b[jj], acc[it][jj]);
        accx[0] = mma4(ax0, bx, accx[0]);
        accx[1] = mma4(ax1, bx, accx[1]);
      }
      if (more) to_lds(buf ^ 1);
      buf ^= 1;
      __syncthreads();
    }
  }
  // ---- slab store: C[i0 + 4 g + r][j0 + c16] ----
  float* out = slab + (size_t)blockIdx.x * KR * FG;
#pragma unroll
  for (int it = 0; it < NI; ++it)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * it + 4 * g + r;
        if (i < KR) out[(size_t)i * FG + 16 * (3 * w + jj) + c16] = acc[it][jj][r];
      }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int it = 2 * w + e;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * it + 4 * g + r;
      if (it < NI && i < KR) out[(size_t)i * FG + 16 * 24 + c16] = accx[e][r];
    }
  }
}

// ------------------------------------------------------------------------------------------
// fp32 weight gradient on the bf16 matrix pipe: three-term split, six products
// ------------------------------------------------------------------------------------------
// lstmf_wgrad_kernel above runs at ~83 % of the fp32 MFMA rate (64 FLOP/clk/SIMD), which is 1/16 of
// the bf16 rate.  Here every fp32 operand a is split EXACTLY into three bf16 terms by truncation,
// a = h + m + l (h = top 8 significand bits, m = the next 8, l = the last 8: the two subtractions
// are exact), and C += A^T D is accumulated as hh + hm + mh + mm + hl + lh on
// v_mfma_f32_16x16x32_bf16 (bf16 x bf16 products are exact in fp32, accumulation in fp32).  The
// dropped terms ml, lm, ll are <= 2^-24 |a b| -- the rounding error of one fp32 product -- so the
// result matches the exact-fp32 kernel to fp32 reduction noise (test_lstmf_wgrad_split_*), at 6/16
// of its matrix-pipe time.
//
// Work split: a workgroup PAIR shares a row range z and splits the 400 gate columns in two parts of
// 208 (13 j-tiles; the second part 192 + 1 zero tile); the pair sits on one XCD (blocks b, b + 8), so
// the A rows [x | h_{t-1} | 1] both read come from the same L2.  Per 32-row chunk the workgroup
// stages the three bf16 planes of A (32 x 208) and of its D part (32 x 208) in LDS, double-buffered
// (2 x 78 KB): the next chunk's fp32 rows are loaded into registers before the MFMAs
// and split into the other buffer after them, one barrier per chunk.  MFMA operands come from
// ds_read_b64_tr_b16 (row-major image, hardware transpose: lane 4q + p of a 16-lane group addresses
// row q, columns 4p..4p+3).  8 waves: wave w owns i-tiles [0, NI0) or [NI0, NI) (w >> 2) times a
// group of 4 / 3 / 3 / 3 local j-tiles (reversed for w >= 4 so each SIMD's two waves carry ~equal
// MFMA counts); its B fragments (all three planes of its <= 3 j-tiles) stay in registers for the
// chunk, the A fragments stream: every operand is read from LDS once per wave.  (A three-part
// column split was measured slower: profiles/r02_split.)
constexpr int WS_CA = 208, WS_CD = 208;                   // max image columns (A, D part)
// Row stride of a plane image with `cols` bf16 columns: S dwords with S % 64 == 8 (cf), else packed.
// One ds_read_b64_tr_b16 lane group (32 lanes) reads 8 consecutive chunk rows (tr_frag's row order) x 8
// dwords; at S % 64 == 8 those are the 64 banks once each.  The r02 stride (416 B = 104 dwords) put
// rows r and r + 8 of the old row order on the same banks: 2-way on every operand read
// (SQ_LDS_BANK_CONFLICT ~ 24 % of the q4 kernel's cycles, profiles/r03_split/pmc_summary_v1.txt).
constexpr int ws_row_bytes(int cols, bool cf) {
  const int dw = (cols + 1) / 2;
  return 4 * (cf ? dw + ((8 - dw % 64) + 64) % 64 : (dw + 3) / 4 * 4);
}
// one double-buffered LDS stage: A image (CA columns) + D image (CD columns), three planes each; the
// conflict-free strides where both buffers fit the 160 KiB
template <int CA, int CD>
struct WImg {
  static constexpr bool CF = 2 * 3 * 32 * (ws_row_bytes(CA, true) + ws_row_bytes(CD, true)) <= 160 * 1024;
  static constexpr int ROWA = ws_row_bytes(CA, CF), ROWD = ws_row_bytes(CD, CF);  // bytes per image row
  static constexpr int PLA = 32 * ROWA, PLD = 32 * ROWD;                           // bytes per plane
  static constexpr int IMGD = 3 * PLA;                                             // D image offset
  static constexpr int BUF = 3 * PLA + 3 * PLD;                                    // one buffer
  static_assert(2 * BUF <= 160 * 1024, "wgrad split LDS");
};
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) char lds_char;
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int KX>
struct WSGeo {
  static constexpr int KR = KX + FH + 1;          // rows of the output slab (bias row last)
  static constexpr int NI = (KR + 15) / 16;       // i-tiles
  static constexpr int NI0 = (NI + 1) / 2;        // i-tiles of waves 0..3
  static constexpr int JX = (32 * KX / 4 + 511) / 512, JH = (32 * FH / 4 + 511) / 512;  // float4 slots per thread
  static constexpr int JD = (32 * 52 + 511) / 512;  // D slots: 52 float4 per row (the second part uses 48)
  static_assert(KX % 4 == 0 && 16 * NI <= WS_CA, "wgrad split: K");
  using Img = WImg<16 * NI, WS_CD>;
};

// three bf16 planes of four fp32 values, packed two per dword (4 VALU per value + 1.5 perms).  Scalar
// on purpose: the pair form (v_pk_add_f32 for the residuals, 4.5 instructions per value) was slower
// beside the MFMAs -- BPTT 7.96 -> 8.34 ms, K = 100 quad weight gradient 14.6 -> 15.4 ms at B = 262 144
// (profiles/r04_ab: gfx950 issues a packed f32 op at more than the cost of two scalar ones).  Plain
// scalars, no ext_vector elements: clang (ROCm 7.2) compiles __builtin_bit_cast(T, vec[i]) / (T, vec.y)
// as a cast of ELEMENT 0 (profiles/r04_ab/README.md; tests/test_isa_hazards.py lints the sources).
__device__ __forceinline__ void split3(const f32x4 v, uint32_t (&p)[3][2]) {
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    uint32_t hb[2], mb[2], lb[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float a = v[2 * e + k];
      const uint32_t u = __builtin_bit_cast(uint32_t, a), h = u & 0xffff0000u;
      const float r1 = a - __builtin_bit_cast(float, h);
      const uint32_t u1 = __builtin_bit_cast(uint32_t, r1), m = u1 & 0xffff0000u;
      const float r2 = r1 - __builtin_bit_cast(float, m);
      hb[k] = h;
      mb[k] = m;
      lb[k] = __builtin_bit_cast(uint32_t, r2);
    }
    // high halves of (x1, x0) -> x0 in the low 16 bits, x1 in the high 16 bits
    p[0][e] = __builtin_amdgcn_perm(hb[1], hb[0], 0x07060302u);
    p[1][e] = __builtin_amdgcn_perm(mb[1], mb[0], 0x07060302u);
    p[2][e] = __builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u);
  }
}

// ---- producer-side split planes ("FP3"): an fp32 tensor (rows, C) stored as its three exact bf16
// split planes, row-planar: row r = [h (C) | m (C) | l (C)] bf16 (6 bytes per value; h + m + l == a
// exactly, so the encoding is lossless and a consumer that loads planes instead of splitting fp32 feeds
// its MFMAs the very same operands: bitwise-identical results).  The gate-column tensors dZ / dZdot
// (C = 400) are stored in the gate-INTERLEAVED column order k = 4 u + q (unit u, gate q) in which the
// split BPTT holds its dz planes; consumers map k back to the natural column (k & 3) H + (k >> 2).
__device__ __forceinline__ constexpr int gate_nat(int k) { return (k & 3) * FH + (k >> 2); }
__device__ __forceinline__ u32x2_t ld8(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(u32x2_t, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}

// fp32 (M, C) -> planes (M, 3, C); IL: column k of the planes is natural column gate_nat(k) (C = 400)
template <bool IL>
__global__ void __launch_bounds__(256) fp3_split_kernel(const float* __restrict__ x, uint16_t* __restrict__ p, int64_t M,
                                                        int C) {
  const int64_t n4 = M * (C / 4);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / (C / 4);
    const int c = 4 * (int)(i - r * (C / 4));
    f32x4 v;
    if constexpr (IL) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = x[r * C + gate_nat(c + j)];
    } else {
      v = *reinterpret_cast<const f32x4*>(x + r * C + c);
    }
    uint32_t q[3][2];
    split3(v, q);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      *reinterpret_cast<u32x2_t*>(p + (r * 3 + pl) * C + c) = u32x2_t{q[pl][0], q[pl][1]};
  }
}
// planes -> fp32 (h + m + l: exact)
template <bool IL>
__global__ void __launch_bounds__(256) fp3_join_kernel(const uint16_t* __restrict__ p, float* __restrict__ x, int64_t M,
                                                       int C) {
  const int64_t n = M * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / C;
    const int k = (int)(i - r * C);
    float a = 0.f;
#pragma unroll
    for (int pl = 2; pl >= 0; --pl) a += __builtin_bit_cast(float, (uint32_t)p[(r * 3 + pl) * C + k] << 16);
    x[r * C + (IL ? gate_nat(k) : k)] = a;
  }
}

// one 16x16x32 operand (8 bf16) of a plane image (row stride ROWB) at column block c0: two
// transposed reads, chunk rows 4 G + q and 16 + 4 G + q of this lane's group G (k = 8 G + j of the
// MFMA maps to chunk row 4 G + j (j < 4) / 16 + 4 G + j - 4: any row order works as long as both
// operands use it; this one keeps a 32-lane read group on 8 consecutive rows); lane_off = the
// lane's (4 G + q) ROWB + 8 p (tr_lane_off)
__device__ __forceinline__ int tr_lane_off(int lane, int rowb) {
  return (4 * (lane >> 4) + ((lane & 15) >> 2)) * rowb + 8 * (lane & 3);
}
template <int ROWB>
__device__ __forceinline__ bf16x8 tr_frag(const lds_char* img, int lane_off, int c0) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + lane_off + c0 * 2));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + lane_off + 16 * ROWB + c0 * 2));
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
__device__ __forceinline__ f32x4 mma32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// one chunk's products for NIV i-tiles x NJV j-tiles of a wave (acc[ii][jj]): the B planes of the
// NJV j-tiles in registers, the A fragments one i-tile ahead.  Each tile's six products go to a
// fresh accumulator that is added to the running sum in VALU fp32 (round to nearest): chaining them
// straight into the running sum on the matrix pipe drifted (3 M rows: 0.043 vs 0.014 for the exact
// kernel, consistent with a biased rounding of the MFMA's C addition).  Straight-line code (one
// instantiation per wave shape): with a wave-uniform branch between an MFMA and the VALU read of its
// result the compiler did not count the wait states across the branch (2 instead of >= 7).
template <class GI, int NIV, int NJV, int NA, int NB>
__device__ __forceinline__ void ws_chunk(f32x4 (&acc)[NA][NB], const lds_char* A_, const lds_char* D_, int tro_a,
                                         int tro_d, int i0, int j0) {
  bf16x8 bfr[NJV][3];
#pragma unroll
  for (int jj = 0; jj < NJV; ++jj)
#pragma unroll
    for (int q = 0; q < 3; ++q) bfr[jj][q] = tr_frag<GI::ROWD>(D_ + q * GI::PLD, tro_d, 16 * (j0 + jj));
#pragma unroll
  for (int ii = 0; ii < NIV; ++ii) {
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 a3[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) a3[q] = tr_frag<GI::ROWA>(A_ + q * GI::PLA, tro_a, 16 * (i0 + ii));
    // j-tiles in pairs: two fresh accumulators in flight, added after both chains
#pragma unroll
    for (int j2 = 0; j2 < NJV; j2 += 2) {
      f32x4 t[2];
#pragma unroll
      for (int jj = j2; jj < j2 + 2 && jj < NJV; ++jj) {
        f32x4& u = t[jj - j2];
        u = mma32(a3[2], bfr[jj][0], f32x4{0.f, 0.f, 0.f, 0.f});  // lh
        u = mma32(a3[0], bfr[jj][2], u);                        // hl
        u = mma32(a3[1], bfr[jj][1], u);                        // mm
        u = mma32(a3[1], bfr[jj][0], u);                        // mh
        u = mma32(a3[0], bfr[jj][1], u);                        // hm
        u = mma32(a3[0], bfr[jj][0], u);                        // hh
      }
#pragma unroll
      for (int jj = j2; jj < j2 + 2 && jj < NJV; ++jj) acc[ii][jj] += t[jj - j2];
    }
  }
}

// XR: X row stride in floats (35: a 36-column image, column 35 zero).  PM: FP3-plane operands as in
// lstmf_wgrad_q4_kernel (bit 1 X -- only with XR == KX --, 2 H, 4 D interleaved)
template <int KX, int XR = KX, int PM = 0>
__global__ void __launch_bounds__(512, 1)
lstmf_wgrad_split_kernel(const void* __restrict__ X, const void* __restrict__ Hs, const void* __restrict__ D,
                         const void* __restrict__ Xd, const void* __restrict__ Hds, const void* __restrict__ Dd,
                         float* __restrict__ slab, int M, int Tn, int rows_per_z, int Z) {
  constexpr bool PX = PM & 1, PH = PM & 2, PD = PM & 4;
  static_assert(!PX || XR == KX, "wgrad split: X planes need XR == KX");
  constexpr int XRB = PX ? 6 * KX : 4 * XR, HRB = PH ? 6 * FH : 4 * FH, DRB = PD ? 6 * FG : 4 * FG;  // row bytes
  using G = WSGeo<KX>;
  using GI = typename G::Img;
  constexpr int NI = G::NI, NI0 = G::NI0, JX = G::JX, JH = G::JH, JD = G::JD;
  extern __shared__ __attribute__((aligned(16))) char wsm_[];
  lds_char* wsm = (lds_char*)wsm_;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // block -> (row range z, column part jh); with Z % 8 == 0 the pair shares an XCD
  int z, jh;
  if (Z % 8 == 0) {
    const int slot = blockIdx.x >> 3;
    jh = slot & 1;
    z = (slot >> 1) * 8 + (blockIdx.x & 7);
  } else {
    jh = blockIdx.x & 1;
    z = blockIdx.x >> 1;
  }
  const int mb = z * rows_per_z, me = min(M, mb + rows_per_z);
  const int jbase = WS_CD * jh, nd4 = jh ? 48 : 52;  // D columns of this part, float4 per row

  // wave tiles: i-half ig, j-group jg (4 / 3 / 3 / 3 of the 13 local j-tiles)
  const int ig = w >> 2, jg = ig ? 3 - (w & 3) : (w & 3);
  const int i0 = ig ? NI0 : 0, ni = ig ? NI - NI0 : NI0;
  const int j0 = jg == 0 ? 0 : 1 + 3 * jg, nj = jg == 0 ? 4 : 3;

  // zero both buffers (pad columns, zero j-tiles of the last part)
  for (int i = tid; i < 2 * GI::BUF / 16; i += 512) reinterpret_cast<__attribute__((address_space(3))) u32x4_t*>(wsm)[i] = u32x4_t{0, 0, 0, 0};
  __syncthreads();

  f32x4 acc[NI0][4];
#pragma unroll
  for (int a = 0; a < NI0; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this lane's transposed-read bases (the D image offset rides in the base VGPR, opaque to the
  // compiler: folded into the reads' immediates it overflowed their 16 bits and cost a register per read)
  const int tro_a = tr_lane_off(lane, GI::ROWA);
  int tro_d = tr_lane_off(lane, GI::ROWD) + GI::IMGD;
  asm volatile("" : "+v"(tro_d));

  // per-thread float4 slots of a 32-row chunk: X (JX), H (JH), D (JD); element e = tid + 512 j:
  // byte offset in the chunk frame (kOOB: none), LDS byte offset (-1: none), H-slot row
  int gx[JX], lx[JX], gh[JH], lh[JH], rhr[JH], gd[JD], ld_[JD], rd_[JD];
#pragma unroll
  for (int j = 0; j < JX; ++j) {
    const int e = tid + 512 * j, r = e / (KX / 4), c4 = e - r * (KX / 4);
    const bool ok = e < 32 * KX / 4;
    gx[j] = ok ? (PX ? r * XRB + 8 * c4 : (r * XR + 4 * c4) * 4) : kOOB;
    lx[j] = ok ? r * GI::ROWA + 8 * c4 : -1;
  }
#pragma unroll
  for (int j = 0; j < JH; ++j) {
    const int e = tid + 512 * j, r = e / (FH / 4), c4 = e - r * (FH / 4);
    const bool ok = e < 32 * FH / 4;
    gh[j] = ok ? (PH ? r * HRB + 8 * c4 : (r * FH + 4 * c4) * 4) : kOOB;
    lh[j] = ok ? r * GI::ROWA + 2 * KX + 8 * c4 : -1;
    rhr[j] = ok ? r : 0;
  }
#pragma unroll
  for (int j = 0; j < JD; ++j) {
    const int e = tid + 512 * j, r = e / 52, c4 = e - r * 52;
    const bool ok = e < 32 * 52 && c4 < nd4;
    gd[j] = ok ? (PD ? r * DRB + 2 * (jbase + 4 * c4) : (r * FG + jbase + 4 * c4) * 4) : kOOB;
    ld_[j] = ok ? GI::IMGD + r * GI::ROWD + 8 * c4 : -1;
    rd_[j] = ok ? r : 0;
  }
  const int step32 = 32 % Tn;

  f32x4 vx[JX], vh[JH], vd[JD];
  u32x2_t px[JX][3], ph[JH][3], pd[JD][3];  // plane slots (dead when the operand is fp32)
  for (int seg = 0; seg < (Xd ? 2 : 1); ++seg) {
    const char* Xs = static_cast<const char*>(seg ? Xd : X);
    const char* Hq = static_cast<const char*>(seg ? Hds : Hs);
    const char* Dq = static_cast<const char*>(seg ? Dd : D);
    // the H descriptor starts at row mb - 1 (row -1 for mb = 0, whose h_{-1} is never addressed: the
    // t = 0 rows are masked) so every voffset is >= 0 -- the range check is on voffset alone, and a
    // negative voffset with a compensating soffset reads zeros
    const int nr = me > mb ? me - mb : 0;
    const rsrc_t rx = make_rsrc(Xs + (size_t)mb * XRB, nr * XRB);
    const rsrc_t rh = make_rsrc(Hq + ((ptrdiff_t)mb - 1) * HRB, (nr ? nr + 1 : 0) * HRB);
    const rsrc_t rd = make_rsrc(Dq + (size_t)mb * DRB, nr * DRB);
    // t = (row) mod Tn of this thread's H slots at the current chunk (h_{-1} = 0 rows)
    int tm[JH];
#pragma unroll
    for (int j = 0; j < JH; ++j) tm[j] = (mb + rhr[j]) % Tn;
    auto load = [&](int m0) {  // rows past me: voffset out of range, zeros
      const int lim = me - m0;
#pragma unroll
      for (int j = 0; j < JX; ++j) {
        if constexpr (PX) {
          const int vo = gx[j] != kOOB && gx[j] / XRB < lim ? gx[j] : kOOB;
#pragma unroll
          for (int q = 0; q < 3; ++q) px[j][q] = ld8(rx, vo + 2 * KX * q, (m0 - mb) * XRB);
        } else {
          vx[j] = ldx4<XR>(rx, (gx[j] >> 2) / XR < lim ? gx[j] : kOOB, (m0 - mb) * XRB, (gx[j] >> 2) % XR);
        }
      }
#pragma unroll
      for (int j = 0; j < JH; ++j) {
        const int vo = rhr[j] < lim && tm[j] != 0 ? gh[j] : kOOB;
        if constexpr (PH) {
#pragma unroll
          for (int q = 0; q < 3; ++q) ph[j][q] = ld8(rh, vo + 2 * FH * q, (m0 - mb) * HRB);
        } else {
          vh[j] = ld4s(rh, vo, (m0 - mb) * HRB);
        }
      }
#pragma unroll
      for (int j = 0; j < JD; ++j) {
        const int vo = rd_[j] < lim ? gd[j] : kOOB;
        if constexpr (PD) {
#pragma unroll
          for (int q = 0; q < 3; ++q) pd[j][q] = ld8(rd, vo + 2 * FG * q, (m0 - mb) * DRB);
        } else {
          vd[j] = ld4s(rd, vo, (m0 - mb) * DRB);
        }
      }
#pragma unroll
      for (int j = 0; j < JH; ++j) {
        tm[j] += step32;
        if (tm[j] >= Tn) tm[j] -= Tn;
      }
    };
    auto put = [&](lds_char* base, int lo, const f32x4& v) {
      if (lo >= 0) {
        uint32_t p[3][2];
        split3(v, p);
        const int pl = lo < GI::IMGD ? GI::PLA : GI::PLD;
#pragma unroll
        for (int q = 0; q < 3; ++q)
          *reinterpret_cast<__attribute__((address_space(3))) u32x2_t*>(base + lo + q * pl) = u32x2_t{p[q][0], p[q][1]};
      }
    };
    auto putp = [&](lds_char* base, int lo, const u32x2_t (&p)[3]) {  // a plane slot: stored as loaded
      if (lo >= 0) {
        const int pl = lo < GI::IMGD ? GI::PLA : GI::PLD;
#pragma unroll
        for (int q = 0; q < 3; ++q) *reinterpret_cast<__attribute__((address_space(3))) u32x2_t*>(base + lo + q * pl) = p[q];
      }
    };
    auto stage = [&](int buf) {
      lds_char* base = wsm + buf * GI::BUF;
#pragma unroll
      for (int j = 0; j < JX; ++j) {
        if constexpr (PX) putp(base, lx[j], px[j]);
        else put(base, lx[j], vx[j]);
      }
#pragma unroll
      for (int j = 0; j < JH; ++j) {
        if constexpr (PH) putp(base, lh[j], ph[j]);
        else put(base, lh[j], vh[j]);
      }
#pragma unroll
      for (int j = 0; j < JD; ++j) {
        if constexpr (PD) putp(base, ld_[j], pd[j]);
        else put(base, ld_[j], vd[j]);
      }
    };
    // bias column (column KR - 1 of A): 1 in plane h for the primal segment, 0 for the tangent one
    if (tid < 64) {
      const int buf = tid >> 5, r = tid & 31;
      *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(wsm + buf * GI::BUF + r * GI::ROWA + (G::KR - 1) * 2) =
          seg ? 0 : 0x3f80;
    }
    const int nch = nr > 0 ? (nr + 31) / 32 : 0;
    if (nch > 0) {
      load(mb);
      stage(0);
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      const bool more = c + 1 < nch;
      if (more) load(mb + 32 * (c + 1));
      const lds_char* A_ = wsm + (c & 1) * GI::BUF;
      const lds_char* D_ = A_;  // (+ IMGD in tro_d)
      switch (ni * 8 + nj) {
        case NI0 * 8 + 4: ws_chunk<GI, NI0, 4>(acc, A_, D_, tro_a, tro_d, i0, j0); break;
        case NI0 * 8 + 3: ws_chunk<GI, NI0, 3>(acc, A_, D_, tro_a, tro_d, i0, j0); break;
        case (NI - NI0) * 8 + 4: ws_chunk<GI, NI - NI0, 4>(acc, A_, D_, tro_a, tro_d, i0, j0); break;
        default: ws_chunk<GI, NI - NI0, 3>(acc, A_, D_, tro_a, tro_d, i0, j0); break;
      }
      if (more) stage((c + 1) & 1);
      __syncthreads();
    }
    __syncthreads();  // (the bias column of both buffers is rewritten for the next segment)
  }
  // slab store: C[16 (i0 + ii) + 4 g + r][jbase + 16 (j0 + jj) + c16]
  float* out = slab + (size_t)z * G::KR * FG;
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int ii = 0; ii < NI0; ++ii)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      if (ii < ni && jj < nj) {
        const int col = jbase + 16 * (j0 + jj) + c16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * (i0 + ii) + 4 * g + r;
          if (i < G::KR && col < FG) out[(size_t)i * FG + (PD ? gate_nat(col) : col)] = acc[ii][jj][r];
        }
      }
}

// ------------------------------------------------------------------------------------------
// split weight gradient, column QUAD: lstmf_wgrad_q4_kernel
// ------------------------------------------------------------------------------------------
// lstmf_wgrad_split_kernel (a workgroup PAIR per row range, 208 columns each) runs its 8 waves in one
// phase at a time -- load -> MFMAs -> split + LDS store -> barrier -- so the matrix pipe idles through
// the split (39.5 % MFMA busy at K = 32), and at K = 100 its 28-tile waves spill (53 ms vs 16 ms
// exact).  Here FOUR workgroups share a row range and split the 400 gate columns in quarters of 100
// (7 j-tiles, the last one 4 / 16 real); the quad sits on one XCD (blocks b, b + 8, b + 16, b + 24),
// so the A rows [x | h_{t-1} | 1] that all four stage come from the same L2.  8 waves (2 per SIMD):
// the NI x 7 output tiles are dealt out as i-groups x j-groups (<= 4 x 4 per wave), so a wave keeps
// its accumulators and <= 2 j-tiles' D fragments in registers and streams the A fragments.
// Prefetch distance two chunks: chunk c + 2's fp32 rows are loaded at the top of chunk c (two
// register sets alternate), and chunk c + 1's rows are split and stored into the other LDS buffer in
// slices between chunk c's i-tiles, so the HBM latency hides under 1.5 chunks of MFMAs and the
// split's VALU issue interleaves with the MFMAs of the same and the partner wave.  Same products and
// accumulation as lstmf_wgrad_split_kernel: six bf16 products per tile into a fresh accumulator,
// added to the running sum in VALU fp32.
constexpr int WQ_CD = 100, WQ_NJ = 7, WQ_W = 8;  // D columns per part, j-tiles per part, waves
template <int KX>
struct WQGeo {
  static constexpr int KR = KX + FH + 1;
  static constexpr int NI = (KR + 15) / 16;
  static constexpr int NIG = (NI + 3) / 4;                  // i-tiles of the first i-group (the rest NI / 4)
  static constexpr int MAXT = NIG * 4;                      // tiles per wave (max): <= 4 i x 4 j
  static constexpr int JX = (32 * KX / 4 + 511) / 512, JH = (32 * FH / 4 + 511) / 512;
  static constexpr int JD = (32 * WQ_CD / 4 + 511) / 512;
  static constexpr int NS = JX + JH + JD;                   // float4 staging slots per thread
  static_assert(KX % 4 == 0 && 16 * NI <= WS_CA && NI <= 16, "wgrad q4: K");
  // wave w: i-group ig, j-group jg (j-tiles 0-3 / 4-6); the two waves of a SIMD (w, w + 4) take
  // mirrored i-groups so the SIMDs carry 25 / 21 / 21 / 24 tiles at K = 100
  static constexpr int ig(int w) { return w < 4 ? w : 3 - (w & 3); }
  static constexpr int i0(int g) { return g == 0 ? 0 : NIG + (g - 1) * ((NI - NIG) / 3) + ((g - 1) < (NI - NIG) % 3 ? g - 1 : (NI - NIG) % 3); }
  static constexpr int ni(int g) { return i0(g + 1 > 3 ? 3 : g + 1) - i0(g) + (g == 3 ? NI - i0(3) : 0); }
  static constexpr int j0(int w) { return w < 4 ? 0 : 4; }
  static constexpr int nj(int w) { return w < 4 ? 4 : 3; }
  using Img = WImg<16 * NI, 16 * WQ_NJ>;
};

// PM: which operands arrive as FP3 planes instead of fp32 (bit 1 X, 2 H, 4 D -- D in the interleaved
// gate order): a plane slot is three 8-byte loads stored to the LDS images as they are, no split
template <int KX, int PM>
__global__ void __launch_bounds__(512, 1)
lstmf_wgrad_q4_kernel(const void* __restrict__ X, const void* __restrict__ Hs, const void* __restrict__ D,
                      const void* __restrict__ Xd, const void* __restrict__ Hds, const void* __restrict__ Dd,
                      float* __restrict__ slab, int M, int Tn, int rows_per_z, int Z) {
  constexpr bool PX = PM & 1, PH = PM & 2, PD = PM & 4;
  constexpr int XRB = PX ? 6 * KX : 4 * KX, HRB = PH ? 6 * FH : 4 * FH, DRB = PD ? 6 * FG : 4 * FG;  // row bytes
  using G = WQGeo<KX>;
  using GI = typename G::Img;
  constexpr int JX = G::JX, JH = G::JH, NS = G::NS, MAXT = G::MAXT;
  extern __shared__ __attribute__((aligned(16))) char wsm_[];
  lds_char* wsm = (lds_char*)wsm_;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // block -> (row range z, column part jq); with Z % 8 == 0 the quad shares an XCD (b, b+8, b+16, b+24)
  int z, jq;
  if (Z % 8 == 0) {
    const int slot = blockIdx.x >> 3;
    jq = slot & 3;
    z = (slot >> 2) * 8 + (blockIdx.x & 7);
  } else {
    jq = blockIdx.x & 3;
    z = blockIdx.x >> 2;
  }
  const int mb = z * rows_per_z, me = min(M, mb + rows_per_z);
  const int jbase = WQ_CD * jq;

  for (int i = tid; i < 2 * GI::BUF / 16; i += 512) reinterpret_cast<__attribute__((address_space(3))) u32x4_t*>(wsm)[i] = u32x4_t{0, 0, 0, 0};
  __syncthreads();

  f32x4 acc[MAXT];
#pragma unroll
  for (int a = 0; a < MAXT; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-buffer lane bases of the transposed reads (A image, D image), opaque to the compiler: with the
  // buffer and image offsets folded into the reads' immediates they overflowed the 16-bit field
  int tro_a[2], tro_d[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    tro_a[b] = tr_lane_off(lane, GI::ROWA) + b * GI::BUF;
    tro_d[b] = tr_lane_off(lane, GI::ROWD) + b * GI::BUF + GI::IMGD;
    asm volatile("" : "+v"(tro_a[b]), "+v"(tro_d[b]));
  }
  const int step32 = 32 % Tn;

  // staging slot s of this thread: kind (x / h / d) is compile-time in s
  auto slot_rc = [&](int s, int& r, int& c4, bool& ok) {
    if (s < JX) {
      const int e = tid + 512 * s;
      r = e / (KX / 4); c4 = e - r * (KX / 4); ok = e < 32 * KX / 4;
    } else if (s < JX + JH) {
      const int e = tid + 512 * (s - JX);
      r = e / (FH / 4); c4 = e - r * (FH / 4); ok = e < 32 * FH / 4;
    } else {
      const int e = tid + 512 * (s - JX - JH);
      r = e / (WQ_CD / 4); c4 = e - r * (WQ_CD / 4); ok = e < 32 * WQ_CD / 4;
    }
    if (!ok) r = c4 = 0;
  };

  f32x4 v[NS];
  u32x2_t pv[NS][3];  // (plane slots; the fp32 / plane element of each slot is dead in the other case)
  for (int seg = 0; seg < (Xd ? 2 : 1); ++seg) {
    const char* Xs = static_cast<const char*>(seg ? Xd : X);
    const char* Hq = static_cast<const char*>(seg ? Hds : Hs);
    const char* Dq = static_cast<const char*>(seg ? Dd : D);
    const int nr = me > mb ? me - mb : 0;
    const rsrc_t rx = make_rsrc(Xs + (size_t)mb * XRB, nr * XRB);
    // (row mb - 1 based: every voffset >= 0; h_{-1} rows are masked by t)
    const rsrc_t rh = make_rsrc(Hq + ((ptrdiff_t)mb - 1) * HRB, (nr ? nr + 1 : 0) * HRB);
    const rsrc_t rd = make_rsrc(Dq + (size_t)mb * DRB + jbase * (PD ? 2 : 4),
                                nr ? (nr - 1) * DRB + (PD ? (2 * FG + WQ_CD) * 2 : WQ_CD * 4) : 0);
    int tm[JH];  // (row mod Tn) of this thread's H slots at the next chunk to load
#pragma unroll
    for (int j = 0; j < JH; ++j) {
      int r, c4;
      bool ok;
      slot_rc(JX + j, r, c4, ok);
      tm[j] = (mb + r) % Tn;
    }
    // slot s of the chunk at row m0 into the register set (rows past me -- or past the range -- read
    // zeros); an H slot's (row mod Tn) then advances to its next chunk
    auto load_slot = [&](int s, int m0) {
      int r, c4;
      bool ok;
      slot_rc(s, r, c4, ok);
      ok = ok && r < me - m0;
      if (s < JX) {
        if constexpr (PX) {
          const int vo = ok ? r * XRB + 8 * c4 : kOOB;
#pragma unroll
          for (int q = 0; q < 3; ++q) pv[s][q] = ld8(rx, vo + 2 * KX * q, (m0 - mb) * XRB);
        } else {
          v[s] = ld4s(rx, ok ? (r * KX + 4 * c4) * 4 : kOOB, (m0 - mb) * XRB);
        }
      } else if (s < JX + JH) {
        int& tmj = tm[s - JX];
        if constexpr (PH) {
          const int vo = ok && tmj != 0 ? r * HRB + 8 * c4 : kOOB;
#pragma unroll
          for (int q = 0; q < 3; ++q) pv[s][q] = ld8(rh, vo + 2 * FH * q, (m0 - mb) * HRB);
        } else {
          v[s] = ld4s(rh, ok && tmj != 0 ? (r * FH + 4 * c4) * 4 : kOOB, (m0 - mb) * HRB);
        }
        tmj += step32;
        if (tmj >= Tn) tmj -= Tn;
      } else {
        if constexpr (PD) {
          const int vo = ok ? r * DRB + 8 * c4 : kOOB;
#pragma unroll
          for (int q = 0; q < 3; ++q) pv[s][q] = ld8(rd, vo + 2 * FG * q, (m0 - mb) * DRB);
        } else {
          v[s] = ld4s(rd, ok ? (r * FG + 4 * c4) * 4 : kOOB, (m0 - mb) * DRB);
        }
      }
    };
    auto stage = [&](lds_char* base, int s) {
      int r, c4;
      bool ok;
      slot_rc(s, r, c4, ok);
      if (!ok) return;
      int lo, pl;
      bool planes;
      if (s < JX) { lo = r * GI::ROWA + 8 * c4; pl = GI::PLA; planes = PX; }
      else if (s < JX + JH) { lo = r * GI::ROWA + 2 * KX + 8 * c4; pl = GI::PLA; planes = PH; }
      else { lo = GI::IMGD + r * GI::ROWD + 8 * c4; pl = GI::PLD; planes = PD; }
      if (planes) {
#pragma unroll
        for (int q = 0; q < 3; ++q) *reinterpret_cast<__attribute__((address_space(3))) u32x2_t*>(base + lo + q * pl) = pv[s][q];
      } else {
        uint32_t p[3][2];
        split3(v[s], p);
#pragma unroll
        for (int q = 0; q < 3; ++q)
          *reinterpret_cast<__attribute__((address_space(3))) u32x2_t*>(base + lo + q * pl) = u32x2_t{p[q][0], p[q][1]};
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    if (tid < 64) {  // bias column KR - 1: 1 in plane h for the primal segment, 0 for the tangent one
      const int buf = tid >> 5, r = tid & 31;
      *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(wsm + buf * GI::BUF + r * GI::ROWA + (G::KR - 1) * 2) =
          seg ? 0 : 0x3f80;
    }
    const int nch = nr > 0 ? (nr + 31) / 32 : 0;
    // prologue: chunk 0 staged into buffer 0, chunk 1 in flight in the register set
#pragma unroll
    for (int s = 0; s < NS; ++s) load_slot(s, mb);
#pragma unroll
    for (int s = 0; s < NS; ++s) stage(wsm, s);
#pragma unroll
    for (int s = 0; s < NS; ++s) load_slot(s, mb + 32);
    __syncthreads();
    // chunk c (S = c & 1): MFMAs on buffer S; between the i-tiles the set's slots (chunk c + 1) are
    // split into buffer S ^ 1, each slot reloaded with chunk c + 2 right after (one register set:
    // a slot's HBM latency hides under one chunk of MFMAs)
    auto chunk = [&](auto S_, int c) {
      constexpr int S = decltype(S_)::value;
      const lds_char* A_ = wsm;  // (+ S BUF in tro_a[S], + S BUF + IMGD in tro_d[S])
      const lds_char* D_ = wsm;
      lds_char* nxt = wsm + (S ^ 1) * GI::BUF;
      // one straight-line body per wave (no branch between an MFMA and the VALU read of its
      // result); wave W owns tiles [TS, TE) of the j-major list (tile L = j NI + i).  The staging
      // slices are unconditional: after the last chunk they store the (zero) rows past the range
      // into the idle buffer
      auto body = [&](auto WK) {
        constexpr int W = decltype(WK)::value;
        constexpr int IG = G::ig(W), I0 = G::i0(IG), NIW = G::ni(IG), J0 = G::j0(W), NJW = G::nj(W);
        constexpr int NJH = (NJW + 1) / 2;                  // j-tiles in pairs: 2 x 3 D fragments held
        constexpr int SPI = (NS + NJH * NIW - 1) / (NJH * NIW);  // staging slots per (pair, i-tile)
        auto jpair = [&](auto JH_) {  // (a lambda per pair: the slot indices below stay compile-time)
          constexpr int jh = decltype(JH_)::value;
          bf16x8 bfr[2][3];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            if (2 * jh + jj < NJW) {
#pragma unroll
              for (int q = 0; q < 3; ++q) bfr[jj][q] = tr_frag<GI::ROWD>(D_ + q * GI::PLD, tro_d[S], 16 * (J0 + 2 * jh + jj));
            }
          // A fragments one i-tile ahead (two sets) where the registers allow (K <= 36): the LDS
          // latency hides under the MFMAs
          constexpr bool PF = KX <= 36;
          bf16x8 af[2][3];
#pragma unroll
          for (int q = 0; q < 3; ++q) af[0][q] = tr_frag<GI::ROWA>(A_ + q * GI::PLA, tro_a[S], 16 * I0);
#pragma unroll
          for (int ii = 0; ii < NIW; ++ii) {
            __builtin_amdgcn_sched_barrier(0);
            if (PF && ii + 1 < NIW) {
#pragma unroll
              for (int q = 0; q < 3; ++q) af[(ii + 1) & 1][q] = tr_frag<GI::ROWA>(A_ + q * GI::PLA, tro_a[S], 16 * (I0 + ii + 1));
            } else if (!PF && ii > 0) {
#pragma unroll
              for (int q = 0; q < 3; ++q) af[ii & 1][q] = tr_frag<GI::ROWA>(A_ + q * GI::PLA, tro_a[S], 16 * (I0 + ii));
            }
            const bf16x8(&a3)[3] = af[ii & 1];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              if (2 * jh + jj >= NJW) continue;  // (compile-time)
              f32x4 t = mma32(a3[2], bfr[jj][0], f32x4{0.f, 0.f, 0.f, 0.f});  // lh
              t = mma32(a3[0], bfr[jj][2], t);                                 // hl
              t = mma32(a3[1], bfr[jj][1], t);                                 // mm
              t = mma32(a3[1], bfr[jj][0], t);                                 // mh
              t = mma32(a3[0], bfr[jj][1], t);                                 // hm
              t = mma32(a3[0], bfr[jj][0], t);                                 // hh
              acc[ii * 4 + 2 * jh + jj] += t;
            }
            const int it = jh * NIW + ii;
#pragma unroll
            for (int s = it * SPI; s < (it + 1) * SPI && s < NS; ++s) {
              stage(nxt, s);
              load_slot(s, mb + 32 * (c + 2));
            }
          }
        };
        jpair(std::integral_constant<int, 0>{});
        if constexpr (NJH > 1) jpair(std::integral_constant<int, 1>{});
      };
      switch (w) {
        case 0: body(std::integral_constant<int, 0>{}); break;
        case 1: body(std::integral_constant<int, 1>{}); break;
        case 2: body(std::integral_constant<int, 2>{}); break;
        case 3: body(std::integral_constant<int, 3>{}); break;
        case 4: body(std::integral_constant<int, 4>{}); break;
        case 5: body(std::integral_constant<int, 5>{}); break;
        case 6: body(std::integral_constant<int, 6>{}); break;
        default: body(std::integral_constant<int, 7>{}); break;
      }
      __syncthreads();
    };
    int c = 0;
    for (; c + 1 < nch; c += 2) {
      chunk(I0{}, c);
      chunk(I1{}, c + 1);
    }
    if (c < nch) chunk(I0{}, c);
    __syncthreads();  // (the bias column of both buffers is rewritten for the next segment)
  }
  // slab store: acc[4 ii + jj] -> C[16 (i0 + ii) + 4 g + r][jbase + 16 (j0 + jj) + c16]
  float* out = slab + (size_t)z * G::KR * FG;
  const int g = lane >> 4, c16 = lane & 15;
  const int igw = G::ig(w), i0w = G::i0(igw), niw = G::ni(igw), j0w = G::j0(w), njw = G::nj(w);
#pragma unroll
  for (int ii = 0; ii < G::NIG; ++ii)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int col = 16 * (j0w + jj) + c16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * (i0w + ii) + 4 * g + r;
        if (ii < niw && jj < njw && i < G::KR && col < WQ_CD)
          out[(size_t)i * FG + (PD ? gate_nat(jbase + col) : jbase + col)] = acc[ii * 4 + jj][r];
      }
    }
}

constexpr int DS_KS = 13;  // the 400 gate columns as 13 k-steps of 32 (k = 400..415 zero)

// ==========================================================================================
// forward / tangent forward with the recurrent product on the bf16 pipe (K <= 36 layers)
// ==========================================================================================
// lstmf_fwd_kernel spends 25 of its 33 k-steps per tile on h_{t-1} U (K = 32: 800 of 1056 MFMA cycles
// per tile and row half on v_mfma_f32_16x16x4_f32).  Here h_{t-1} U runs as the exact three-term split
// (h = h_h + h_m + h_l, U = U_h + U_m + U_l by truncation, six products lh + hl + mm + mh + hm + hh on
// v_mfma_f32_16x16x32_bf16, dropped terms <= 2^-24 of each product) over k = 0..95 and exactly in fp32
// for k = 96..99 (one 16x16x4 k-step): 3 x 6 x 16 + 32 = 320 instead of 800 cycles per tile and row
// half.  The split products chain into the exact-fp32 x W accumulator.  U's planes (3 k-steps x 7 tiles x 3 planes, 252 registers) are pinned in AGPRs; h_{t-1} lives
// in LDS as three bf16 planes [32 rows][104] (row stride: conflict-free ds_read_b128) plus an fp32
// tail [32][4]; the cell update writes its h (or hdot) straight into them.  Everything else -- the
// gate-interleaved tiles, the quad transpose, the tapes, x W on the exact fp32 MFMA -- is
// lstmf_fwd_kernel's.
// Plane row strides for the 16x16x32 A-fragment ds_read_b128 (lane l: row l & 15, k-group l >> 4, i.e.
// dword S (l & 15) + 4 (l >> 4)): conflict-free over the CDNA4 b128 lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} (+32) only for S = 56, 72 (mod 64 multiples) / 216, 232, 248 dwords; the r03 strides
// (52 / 212 dwords) were conflict-free for contiguous 16-lane groups only and 2-way on the real ones
// (bwds: SQ_LDS_BANK_CONFLICT 1.56x its LDS-active cycles, profiles/r03_bwds/pmc_bptt_B262144.txt)
constexpr int FS_HR = 112;                                // h plane row stride (bf16 elements): 56 dwords
constexpr int FS_HPL = 32 * FS_HR * 2;                    // bytes per h plane (32 rows)
constexpr int FS_HB = 3 * FS_HPL + 32 * 4 * 4;            // one h buffer: 3 planes + fp32 tail [32][4]

__device__ __forceinline__ uint32_t trunc_hi(float a) { return __builtin_bit_cast(uint32_t, a) & 0xffff0000u; }

template <int ACT, int KX, bool TAPE, bool TAN>
__global__ void __launch_bounds__(256, 1)
lstmf_fwds_kernel(const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                  const float* __restrict__ U, const float* __restrict__ ptape, float* __restrict__ hs,
                  float* __restrict__ tape, int B, int Tn) {
  using GX = FGeo<KX>;
  static_assert(GX::KS <= 12, "split forward: K <= 48 (W^T in registers)");
  constexpr int NW = GX::KS;
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  float* xb = fsm;                                                  // [2][32 * LRX] fp32, K-permuted
  float* trash = xb + 2 * 32 * GX::LR;                              // [4] padding / out-of-range writes
  lds_char* trashc = (lds_char*)trash;
  lds_char* hb = (lds_char*)(trash + 4);                            // [2][FS_HB] h planes + tail
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane & 3, g = lane >> 4, j4 = (lane & 15) >> 2;
  const int ub = FUW * w + j4;
  const int nrb = (B + 31) / 32;

  for (int i = tid; i < 2 * 32 * GX::LR; i += 256) xb[i] = 0.f;

  constexpr float GSC = ACT == ACT_TANH ? -2.f * kLog2e : ACT == ACT_SIGMOID ? -kLog2e : 1.f;
  const float sc = TAN ? 1.f : (q == 2 ? GSC : -kLog2e);
  // B operands.  16x16x32: lane l holds B[k = 32 ks + 8 (l >> 4) + j][col l & 15] (j < 8); the fp32
  // tail 16x16x4: B[k = 96 + (l >> 4)][col]; x W (16x16x4): B[k = 4 ks + (l >> 4)][col]
  bf16x8 up[3][FNT][3];
  float ut[FNT], wf[NW][FNT], bq[FNT];
#pragma unroll
  for (int n = 0; n < FNT; ++n) {
    const int u = ub + 4 * n;
    const bool ok = u < FH;
    const int cl = q * FH + (ok ? u : FH - 1);
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      uint32_t hh[8], mm[8], ll[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * ks + 8 * g + j;  // < 96
        const float v = ok ? U[k * FG + cl] * sc : 0.f;
        const uint32_t h = trunc_hi(v);
        const float r1 = v - __builtin_bit_cast(float, h);
        const uint32_t m = trunc_hi(r1);
        const float r2 = r1 - __builtin_bit_cast(float, m);
        hh[j] = h; mm[j] = m; ll[j] = __builtin_bit_cast(uint32_t, r2);
      }
      uint4 ph, pm, pl;
      ph.x = __builtin_amdgcn_perm(hh[1], hh[0], 0x07060302u); ph.y = __builtin_amdgcn_perm(hh[3], hh[2], 0x07060302u);
      ph.z = __builtin_amdgcn_perm(hh[5], hh[4], 0x07060302u); ph.w = __builtin_amdgcn_perm(hh[7], hh[6], 0x07060302u);
      pm.x = __builtin_amdgcn_perm(mm[1], mm[0], 0x07060302u); pm.y = __builtin_amdgcn_perm(mm[3], mm[2], 0x07060302u);
      pm.z = __builtin_amdgcn_perm(mm[5], mm[4], 0x07060302u); pm.w = __builtin_amdgcn_perm(mm[7], mm[6], 0x07060302u);
      pl.x = __builtin_amdgcn_perm(ll[1], ll[0], 0x07060302u); pl.y = __builtin_amdgcn_perm(ll[3], ll[2], 0x07060302u);
      pl.z = __builtin_amdgcn_perm(ll[5], ll[4], 0x07060302u); pl.w = __builtin_amdgcn_perm(ll[7], ll[6], 0x07060302u);
      up[ks][n][0] = __builtin_bit_cast(bf16x8, ph);
      up[ks][n][1] = __builtin_bit_cast(bf16x8, pm);
      up[ks][n][2] = __builtin_bit_cast(bf16x8, pl);
#pragma unroll
      for (int p = 0; p < 3; ++p) asm volatile("" : "+a"(up[ks][n][p]));
    }
    ut[n] = ok ? U[(96 + g) * FG + cl] * sc : 0.f;
#pragma unroll
    for (int ks = 0; ks < NW; ++ks) {
      const int k = 4 * ks + g;
      const float v = W[min(k, KX - 1) * FG + cl];
      wf[ks][n] = (ok && k < KX) ? v * sc : 0.f;
    }
    const float bv = bias ? bias[cl] : 0.f;
    bq[n] = (!TAN && ok) ? bv * sc : 0.f;
  }
  const bool glin = !TAN && ACT == ACT_LINEAR && q == 2;
  const float am = (ACT == ACT_TANH && q == 2) ? 2.f : 1.f, bm = (ACT == ACT_TANH && q == 2) ? -1.f : 0.f;
  const int ax = (lane & 15) * GX::LR + g * GX::KQ;
  // this lane's h fragments: plane row (lane & 15) (+ 16 m), k = 32 ks + 8 g; tail row, k = 96 + g
  const int ahp = ((lane & 15) * FS_HR + 8 * g) * 2, aht = 3 * FS_HPL + ((lane & 15) * 4 + g) * 4;

  for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
    const int row0 = rb * 32;
    const rsrc_t rx = ftile_rsrc(x, row0, B, Tn, KX);
    const rsrc_t rh = ftile_rsrc(hs, row0, B, Tn, FH);
    const rsrc_t rt = ftape_rsrc(TAPE ? tape : nullptr, rb, nrb, Tn);
    const rsrc_t rp = ftape_rsrc(TAN ? ptape : nullptr, rb, nrb, Tn);
    int vp1[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) vp1[m] = ((16 * m + 4 * g + q) * Tn * FH + ub) * 4;
    const int tl = ftape_lane(w, lane), tcl = ftape_cell(w, lane);
    float cprev[TAN ? 2 : 1][FNT];
    if constexpr (TAN) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < FNT; ++n) cprev[m][n] = 0.f;
    }
    float cst[2][FNT];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < FNT; ++n) cst[m][n] = 0.f;
    FXPart<KX> xp;
    xp.set(Tn, tid);
    xp.load(rx, Tn, 0, true);
    // h_{-1} = 0: buffer 0 planes + tail
    for (int i = tid; i < FS_HB / 16; i += 256)
      reinterpret_cast<__attribute__((address_space(3))) u32x4_t*>(hb)[i] = u32x4_t{0, 0, 0, 0};
    xp.to_lds(xb, trash);
    __syncthreads();
    for (int t = 0; t < Tn; ++t) {
      const float* xcur = xb + (t & 1) * 32 * GX::LR;
      const lds_char* hcur = hb + (t & 1) * FS_HB;
      lds_char* hnext = hb + ((t + 1) & 1) * FS_HB;
      xp.load(rx, Tn, t + 1, t + 1 < Tn);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        f32x4 pg[TAN ? FNT : 1];
        float pc[TAN ? FNT : 1];
        const int p1 = vp1[m] + t * FH * 4, tb = t * FT_STEP * 4;
        if constexpr (TAN) {
#pragma unroll
          for (int n = 0; n < FNT; ++n) {
            const bool tok = !(w == 3 && n >= 4);
            pg[n] = ld4(rp, tok ? tl + tb + ftape_slot(m, n) : kOOB);
            pc[n] = ld1(rp, tok ? tcl + tb + ftape_slot(m, n) : kOOB, 0);
          }
        }
        f32x4 acc[FNT];
#pragma unroll
        for (int n = 0; n < FNT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        // ---- z = x_t W (exact fp32) ----
#pragma unroll
        for (int j = 0; j < GX::NJ; ++j) {
          const f32x4 a4 = *reinterpret_cast<const f32x4*>(xcur + ax + 16 * m * GX::LR + 4 * j);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int ks = 4 * j + s4;
            if (ks >= GX::KS) break;
#pragma unroll
            for (int n = 0; n < FNT; ++n) acc[n] = mma4(a4[s4], wf[ks][n], acc[n]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        // ---- + h_{t-1} U: the split k < 96 and the exact fp32 tail, chained into acc (20 accumulation
        // steps per element: the MFMA C-addition rounding stays at the fp32 noise level here) ----
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
          const lds_char* ar = hcur + ahp + 16 * m * FS_HR * 2 + 64 * ks;
          const bf16x8 a0 = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(ar);
          const bf16x8 a1 = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(ar + FS_HPL);
          const bf16x8 a2 = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(ar + 2 * FS_HPL);
#pragma unroll
          for (int n = 0; n < FNT; ++n) {
            f32x4 t6 = acc[n];
            t6 = mma32(a2, up[ks][n][0], t6);  // lh
            t6 = mma32(a0, up[ks][n][2], t6);  // hl
            t6 = mma32(a1, up[ks][n][1], t6);  // mm
            t6 = mma32(a1, up[ks][n][0], t6);  // mh
            t6 = mma32(a0, up[ks][n][1], t6);  // hm
            acc[n] = mma32(a0, up[ks][n][0], t6);  // hh
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        {
          const float at = *reinterpret_cast<const __attribute__((address_space(3))) float*>(hcur + aht + 16 * m * 16);
#pragma unroll
          for (int n = 0; n < FNT; ++n) acc[n] = mma4(at, ut[n], acc[n]);
        }
        // ---- gate math, cell update, stores (row 16 m + 4 g + q, unit ub + 4 n after the transpose) ----
#pragma unroll
        for (int n = 0; n < FNT; ++n) {
          const bool tok = !(w == 3 && n >= 4);  // wave 3's tiles 4..6 are padding units 100..111
          const int v1 = tok ? p1 + 16 * n : kOOB;
          const f32x4 zs = acc[n];
          float hv;
          if constexpr (!TAN) {
            float y[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float s_ = zs[i] + bq[n];
              const float e = am * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(s_)) + bm;
              y[i] = glin ? s_ : e;
            }
            quad_transpose(y, q);
            const float cn = y[1] * cst[m][n] + y[0] * y[2];
            float ca;
            if constexpr (ACT == ACT_TANH) ca = 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(GSC * cn)) - 1.f;
            else if constexpr (ACT == ACT_SIGMOID) ca = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(GSC * cn));
            else ca = cn;
            hv = tok ? y[3] * ca : 0.f;
            cst[m][n] = cn;
            if constexpr (TAPE) {
              st4(f32x4{y[0], y[1], y[2], y[3]}, rt, tok ? tl + tb + ftape_slot(m, n) : kOOB);
              st1(cn, rt, tok ? tcl + tb + ftape_slot(m, n) : kOOB, 0);
            }
          } else {
            float zd[4] = {zs[0], zs[1], zs[2], zs[3]};
            quad_transpose(zd, q);
            const f32x4 y = pg[n];
            const float idot = y[0] * (1.f - y[0]) * zd[0], fdot = y[1] * (1.f - y[1]) * zd[1];
            const float gdot = act_dy(ACT, y[2]) * zd[2], odot = y[3] * (1.f - y[3]) * zd[3];
            const float c = pc[n];
            float cdn = fdot * cprev[m][n] + y[1] * cst[m][n] + idot * y[2] + y[0] * gdot;
            const float ca = act_f(ACT, c);
            float hd = odot * ca + y[3] * act_dy(ACT, ca) * cdn;
            if (!tok) { cdn = 0.f; hd = 0.f; }
            cst[m][n] = cdn;
            cprev[m][n] = c;
            hv = hd;
            st4(f32x4{zd[0], zd[1], zd[2], zd[3]}, rt, tok ? tl + tb + ftape_slot(m, n) : kOOB);
            st1(cdn, rt, tok ? tcl + tb + ftape_slot(m, n) : kOOB, 0);
          }
          // h (or hdot) of (row 16 m + 4 g + q, unit u) into the next step's planes / tail; units
          // >= 100 (wave 3's padding tiles) go to the trash word
          {
            const int u = ub + 4 * n, row = 16 * m + 4 * g + q;
            const uint32_t h1 = trunc_hi(hv);
            const float r1 = hv - __builtin_bit_cast(float, h1);
            const uint32_t m1 = trunc_hi(r1);
            const uint32_t l1 = __builtin_bit_cast(uint32_t, r1 - __builtin_bit_cast(float, m1));
            const bool pl = u < 96;
            lds_char* dp = pl ? hnext + (row * FS_HR + u) * 2 : trashc;
            *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(dp) = (uint16_t)(h1 >> 16);
            *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(dp + (pl ? FS_HPL : 0)) = (uint16_t)(m1 >> 16);
            *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(dp + (pl ? 2 * FS_HPL : 0)) = (uint16_t)(l1 >> 16);
            const bool tl4 = u >= 96 && u < FH;
            lds_char* tp = tl4 ? hnext + 3 * FS_HPL + (row * 4 + (u - 96)) * 4 : trashc;
            *reinterpret_cast<__attribute__((address_space(3))) float*>(tp) = hv;
          }
          st1(hv, rh, v1, 0);
        }
      }
      xp.to_lds(xb + ((t + 1) & 1) * 32 * GX::LR, trash);
      lds_barrier();
    }
  }
}

// ------------------------------------------------------------------------------------------
// BPTT with the recurrent product on the bf16 matrix pipe: lstmf_bwds_kernel
// ------------------------------------------------------------------------------------------
// lstmf_bwdp_kernel's step is bound by dh_rec = dz_{t+1} U^T on the exact fp32 MFMA (400 16x16x4
// MFMAs per MFMA-role wave and step).  Here the product is the exact three-term bf16 split (dz and U^T
// each h + m + l; six products lh hl mm mh hm hh, the dropped terms <= 2^-24 of each product) on
// v_mfma_f32_16x16x32_bf16: 13 k-steps x 2 tiles x 6 = 156 MFMAs per half tile and wave, ~1/2.5 of the
// fp32 pipe time.  The matrix work and the cell math are then of the same size, so the roles merge:
// 4 waves (one per SIMD, 512 registers), wave w does the MFMAs of output tiles 2 w, 2 w + 1 AND the
// cells of units 28 w .. 28 w + 27, one cell after each of the first 7 k-steps, so the VALU issues the
// cell math of one row half while the matrix pipe runs the other half's product.  The row-half pipeline
// is lstmf_bwdp_kernel's:
//   P1(t): B(0, t) + A(1, t)      P2(t): B(1, t) + A(0, t - 1)
// The dz tile has two images: the fp32 rows (dZ's coalesced HBM stores, as before) and three bf16
// planes in the gate-interleaved column order k = 4 u + q (a cell writes its four gates as one 8-byte
// word per plane), row stride 424 (conflict-free ds_read_b128).  B[k][j] = U[j][(k & 3) H + (k >> 2)],
// k >= 400 zero: 312 registers per wave, 252 of them pinned in AGPRs.  One tape register set: a cell's
// loads for the other half's next use are issued as soon as it has consumed the set.
constexpr int BS_LZ = 432;             // dz plane row stride (bf16 elements): 216 dwords
constexpr int BS_PL = 32 * BS_LZ * 2;  // bytes per dz plane (32 rows)

template <int ACT, bool HEAD = false>
__global__ void __launch_bounds__(256, 1)
lstmf_bwds_kernel(const float* __restrict__ dH, const float* __restrict__ tape, const float* __restrict__ U,
                  float* __restrict__ dZ, int B, int Tn, const float* __restrict__ hd, const float* __restrict__ hw) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  float* zt = fsm;                                     // fp32 dz tile [32][BZ_LR]: [q][u'] per row
  float* ht = zt + 32 * BZ_LR;                         // dh_rec tile [32][BH_LR]
  float* trash = ht + 32 * BH_LR;                      // [4 * BZ_KQ + 4] padding words, never read
  lds_char* trashp = (lds_char*)(trash + 4 * BZ_KQ);
  lds_char* zp = (lds_char*)(trash + 4 * BZ_KQ + 4);   // dz planes [3][32][BS_LZ] bf16
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane & 3, g = lane >> 4, j4 = (lane & 15) >> 2, c16 = lane & 15;
  const int nrb = (B + 31) / 32;
  // U^T planes: B[k = 32 ks + 8 g + j][col 16 (2 w + e) + c16] = U[col][(k & 3) H + (k >> 2)]
  bf16x8 up[2][DS_KS][3];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int col = 16 * (2 * w + e) + c16;
    const bool ok = col < FH;
#pragma unroll
    for (int ks = 0; ks < DS_KS; ++ks) {
      f32x4 v[2];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = min(32 * ks + 8 * g + j, FG - 1);
        const float x = U[(ok ? col : 0) * FG + (k & 3) * FH + (k >> 2)];
        v[j >> 2][j & 3] = (ok && 32 * ks + 8 * g + j < FG) ? x : 0.f;
      }
      uint32_t p0[3][2], p1[3][2];
      split3(v[0], p0);
      split3(v[1], p1);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        up[e][ks][p] = __builtin_bit_cast(bf16x8, make_uint4(p0[p][0], p0[p][1], p1[p][0], p1[p][1]));
        if (e == 1 || ks < 8) asm volatile("" : "+a"(up[e][ks][p]));
      }
    }
  }
  const int ub = FUW * w + j4;
  const int hr = (4 * g + q) * BH_LR + ub, zw = (4 * g + q) * BZ_LR + ub;  // (+16 m rows, + 4 n units)
  const int zpw = ((4 * g + q) * BS_LZ + 4 * ub) * 2;                    // plane word (+ 32 n bytes)
  const int ao = (c16 * BS_LZ + 8 * g) * 2;  // A fragment: row c16 (+ 16 M), k = 32 ks + 8 g .. + 7
  // dZ store share: threads 0..199 own chunk tid % 100 of rows 2 k + tid / 100 (k < 16)
  const int srr = tid / 100, sch = tid - 100 * srr, sqq = sch / 25, sc = sch - 25 * sqq;
  const int slo = (srr & 1) * BZ_LR + sqq * BZ_KQ + 4 * sc;
  const int sgo = tid < 200 ? (srr * Tn * FG + sqq * FH + 4 * sc) * 4 : kOOB;
  const int tl = ftape_lane(w, lane), tcl = ftape_cell(w, lane);
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
    const int row0 = rb * 32;
    const rsrc_t rdh = ftile_rsrc(dH, row0, B, Tn, FH), rt = ftape_rsrc(tape, rb, nrb, Tn);
    const rsrc_t rz = ftile_rsrc(dZ, row0, B, Tn, FG);
    const int nr = min(32, B - row0);
    int vp1[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) vp1[m] = ((16 * m + 4 * g + q) * Tn * FH + ub) * 4;
    // HEAD: the lane rows' head adjoint factors d[row] (0 past B) and the head weight's descriptor
    float hdv[2] = {0.f, 0.f};
    const rsrc_t rhw = make_rsrc(hw, HEAD ? Tn * FH * 4 : 0);
    if constexpr (HEAD) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int r = row0 + 16 * m + 4 * g + q;
        hdv[m] = r < B ? hd[r] : 0.f;
      }
    }
    const int hvo = ub * 4;
    float dc[2][FNT], tc[2][FNT];
    f32x4 tg[FNT];
    float tcp[FNT], tdh[FNT];
    const int T1 = Tn - 1;
#pragma unroll
    for (int n = 0; n < FNT; ++n) {
      const bool tok = !(w == 3 && n >= 4);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        dc[m][n] = 0.f;
        tc[m][n] = ld1(rt, tok ? tcl + T1 * FT_STEP * 4 + ftape_slot(m, n) : kOOB, 0);  // c_{T-1}
      }
      bwdf_tape_load_u<HEAD>(tg[n], tcp[n], tdh[n], rt, rdh, tl, tcl, vp1[0], T1 * FT_STEP * 4 + ftape_slot(0, n),
                             max(T1 - 1, 0) * FT_STEP * 4 + ftape_slot(0, n), T1 * FH * 4 + 16 * n, tok, T1 > 0, hdv[0],
                             rhw, hvo);
    }
    // dz_T = 0 (planes, pad columns k >= 400 included), dh_rec(T - 1) = 0
    for (int i = tid; i < 3 * BS_PL / 16; i += 256)
      reinterpret_cast<__attribute__((address_space(3))) u32x4_t*>(zp)[i] = u32x4_t{0, 0, 0, 0};
    for (int i = tid; i < 32 * BH_LR; i += 256) ht[i] = 0.f;
    __syncthreads();
    // rows of half M of the fp32 dz tile (dz at step ts) -> dZ[:, ts, :]
    auto store_half = [&](auto M_, int ts) {
      constexpr int M = decltype(M_)::value;
#pragma unroll
      for (int k = 8 * M; k < 8 * M + 8; ++k) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(zt + slo + 2 * k * BZ_LR);
        st16(v, rz, 2 * k + srr < nr, sgo, (2 * k * Tn + ts) * FG * 4);
      }
    };
    // cell adjoint of (row half M, unit tile n) at step t, then the loads for the set's next use
    auto cell = [&](auto M_, int n, float hrec, int t) {
      constexpr int m = decltype(M_)::value;
      const bool tok = !(w == 3 && n >= 4);
      const float ig = tg[n][0], fg = tg[n][1], gg = tg[n][2], og = tg[n][3];
      const float dht = tdh[n] + hrec;
      const float ca = act_f(ACT, tc[m][n]);
      const float dov = dht * ca;
      const float dct = dc[m][n] + dht * og * act_dy(ACT, ca);
      dc[m][n] = tok ? dct * fg : 0.f;
      f32x4 z4;
      z4[0] = dct * gg * ig * (1.f - ig);
      z4[1] = dct * tcp[n] * fg * (1.f - fg);
      z4[2] = dct * ig * act_dy(ACT, gg);
      z4[3] = dov * og * (1.f - og);
      float* zd = tok ? zt + zw + 16 * m * BZ_LR + 4 * n : trash;
#pragma unroll
      for (int k = 0; k < 4; ++k) zd[k * BZ_KQ] = z4[k];
      uint32_t p[3][2];
      split3(z4, p);
      lds_char* pd = tok ? zp + zpw + 16 * m * BS_LZ * 2 + 32 * n : trashp;
      const int ps = tok ? BS_PL : 0;
#pragma unroll
      for (int pp = 0; pp < 3; ++pp)
        *reinterpret_cast<__attribute__((address_space(3))) u32x2_t*>(pd + pp * ps) = u32x2_t{p[pp][0], p[pp][1]};
      tc[m][n] = tcp[n];  // c_{t-1} is the next step's c
      if constexpr (m == 0) {  // next use: B(1, t)
        bwdf_tape_load_u<HEAD>(tg[n], tcp[n], tdh[n], rt, rdh, tl, tcl, vp1[1], t * FT_STEP * 4 + ftape_slot(1, n),
                               max(t - 1, 0) * FT_STEP * 4 + ftape_slot(1, n), t * FH * 4 + 16 * n, tok, t > 0, hdv[1],
                               rhw, hvo);
      } else {  // next use: B(0, t - 1)
        const int tp = t > 0 ? t - 1 : 0;
        bwdf_tape_load_u<HEAD>(tg[n], tcp[n], tdh[n], rt, rdh, tl, tcl, vp1[0], tp * FT_STEP * 4 + ftape_slot(0, n),
                               max(tp - 1, 0) * FT_STEP * 4 + ftape_slot(0, n), tp * FH * 4 + 16 * n, tok && t > 0,
                               tp > 0, hdv[0], rhw, hvo);
      }
    };
    // one half-phase: dz rows of half MA out to HBM, the cells of half 1 - MA at step t, and rows MA of
    // dh_rec = dz[rows MA] U^T (the planes hold dz_{t + 1} there for MA = 1, dz_t for MA = 0)
    auto phase = [&](auto MA_, int t) {
      constexpr int MA = decltype(MA_)::value;
      if constexpr (MA == 1) {
        if (t < T1) store_half(I1{}, t + 1);
      } else {
        store_half(I0{}, t);
      }
      float hv[FNT];  // the cells' dh_rec words (rows of half 1 - MA, completed in the previous phase)
#pragma unroll
      for (int n = 0; n < FNT; ++n) hv[n] = ht[hr + 16 * (1 - MA) * BH_LR + 4 * n];
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      const lds_char* ar = zp + ao + 16 * MA * BS_LZ * 2;
      bf16x8 af[2][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) af[0][p] = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(ar + p * BS_PL);
#pragma unroll
      for (int ks = 0; ks < DS_KS; ++ks) {
        if (ks + 1 < DS_KS) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            af[(ks + 1) & 1][p] = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(ar + p * BS_PL + 64 * (ks + 1));
        }
        const bf16x8(&a)[3] = af[ks & 1];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          acc[e] = mma32(a[2], up[e][ks][0], acc[e]);  // lh
          acc[e] = mma32(a[0], up[e][ks][2], acc[e]);  // hl
          acc[e] = mma32(a[1], up[e][ks][1], acc[e]);  // mm
          acc[e] = mma32(a[1], up[e][ks][0], acc[e]);  // mh
          acc[e] = mma32(a[0], up[e][ks][1], acc[e]);  // hm
          acc[e] = mma32(a[0], up[e][ks][0], acc[e]);  // hh
        }
        if (ks < FNT) cell(std::integral_constant<int, 1 - MA>{}, ks, hv[ks], t);  // (compile-time)
      }
      // one schedule for the whole phase: per k-step its A fragments, then its 12 MFMAs with 3 VALU
      // slots (the cells' math) after each one; loads and LDS stores of the cells go where they fit
#pragma unroll
      for (int ks = 0; ks < DS_KS; ++ks) {
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // rows 16 MA + 4 g + i, column 16 (2 w + e) + c16 (wave 3's second tile is past the 112 units: trash)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool ok = 2 * w + e < 7;
        float* hd = ok ? ht + (16 * MA + 4 * g) * BH_LR + 16 * (2 * w + e) + c16 : trash;
        const int hs = ok ? BH_LR : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) hd[i * hs] = acc[e][i];
      }
      lds_barrier();
    };
    for (int t = T1; t >= 0; --t) {
      phase(I1{}, t);  // P1(t): B(0, t) + A(1, t)
      phase(I0{}, t);  // P2(t): B(1, t) + A(0, t - 1)
    }
    store_half(I1{}, 0);
    __syncthreads();  // (the tiles are re-zeroed for the next row block)
  }
}

// ------------------------------------------------------------------------------------------
// fp32 input gradient on the bf16 matrix pipe, LDS-staged: lstmf_dgrad_s4_kernel
// ------------------------------------------------------------------------------------------
// dX = dZ W^T with the exact three-term split (six products, dropped terms <= 2^-24 of each product).
// lstmf_dgrad_split_kernel splits the 400-long reduction across its 8 waves and reduces their partial
// tiles in LDS per 16-row tile (barrier + 8-way sum per tile: slower than the exact kernel).  Here the
// reduction stays inside one wave: 4 waves (one per SIMD, 512-register budget), wave w owns output
// columns 32 w .. 32 w + 31 (two 16-column tiles) and holds the three W^T planes of BOTH tiles and ALL 13
// k-steps (k = 400..415 zero) in registers (312 VGPRs).  The 16-row dZ chunks are fp32-loaded two chunks
// ahead (two register sets), split into the three bf16 planes and stored to a double-buffered LDS image
// (row stride 424 elements: conflict-free ds_read_b128 A fragments) in slices between the second half
// of the k-steps, so the split's VALU issue interleaves with the wave's MFMAs.  One barrier per chunk;
// each chunk's output tiles are final (no partial tiles, no cross-wave reduction).
constexpr int DS4_RS = 432;                   // LDS image row stride (bf16 elements): >= 416, conflict-free b128
constexpr int DS4_PL = 16 * DS4_RS * 2;       // bytes per plane image (16 rows)
constexpr int DS4_BUF = 3 * DS4_PL;           // one buffer: three planes
constexpr int DS4_SLOTS = (16 * 100 + 255) / 256;  // float4 staging slots per thread per chunk (7)
constexpr int DS4_K0 = DS_KS - DS4_SLOTS;     // first k-step followed by a staging slot
// register sets of the dZ prefetch: 2 = one chunk ahead (three sets, two chunks ahead, measured
// 3.59 vs 3.54 ms at 6.3 M rows: profiles/r04_wgrad/wdma2)
constexpr int DS4_NS = 2;

// PD: dZ arrives as FP3 planes in the interleaved gate order (W^T's k runs over gate_nat(k) then, and the
// staging copies the planes as loaded: no split)
template <int NT2, bool PD = false>
__global__ void __launch_bounds__(256, 1)
lstmf_dgrad_s4_kernel(const void* __restrict__ D, const float* __restrict__ W, float* __restrict__ X, int M, int KO) {
  constexpr int DRB = PD ? 6 * FG : 4 * FG;  // dZ row bytes
  extern __shared__ __attribute__((aligned(16))) char dsm_[];
  lds_char* dsm = (lds_char*)dsm_;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int nch = (M + 15) / 16;
  // W^T planes of output tiles 2 w + e: B[k = 32 ks + 8 g + j][col 16 (2 w + e) + c16] = W[col][k]
  bf16x8 bw[2][DS_KS][3];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int col = 16 * (2 * w + e) + c16;
#pragma unroll
    for (int ks = 0; ks < DS_KS; ++ks) {
      const int k0 = 32 * ks + 8 * g;
      f32x4 v0 = f32x4{0.f, 0.f, 0.f, 0.f}, v1 = v0;
      if (w < NT2 && col < KO && k0 < FG) {
        if constexpr (PD) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v0[j] = W[(size_t)col * FG + gate_nat(k0 + j)];
            v1[j] = W[(size_t)col * FG + gate_nat(k0 + 4 + j)];
          }
        } else {
          v0 = *reinterpret_cast<const f32x4*>(W + (size_t)col * FG + k0);
          v1 = *reinterpret_cast<const f32x4*>(W + (size_t)col * FG + k0 + 4);
        }
      }
      uint32_t p0[3][2], p1[3][2];
      split3(v0, p0);
      split3(v1, p1);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        bw[e][ks][q] = __builtin_bit_cast(bf16x8, make_uint4(p0[q][0], p0[q][1], p1[q][0], p1[q][1]));
        // tile 1's planes live in the accumulator half of the register file (MFMA B operands may be
        // AGPRs): without the pin the compiler parks them there anyway and copies each one back to
        // VGPRs before its MFMA (4 v_accvgpr_read per MFMA)
        if (e == 1) asm volatile("" : "+a"(bw[e][ks][q]));
      }
    }
  }
  f32x4 v[DS4_NS][DS4_SLOTS];
  u32x2_t pv[DS4_NS][DS4_SLOTS][3];  // (PD)
  auto load = [&](auto S_, int c) {  // chunk c's rows (past M: zero-size descriptor, zeros)
    constexpr int S = decltype(S_)::value;
    const int r0 = c * 16, nr = c < nch ? min(16, M - r0) : 0;
    const rsrc_t rd = make_rsrc(static_cast<const char*>(D) + (nr ? (size_t)r0 * DRB : 0), nr * DRB);
#pragma unroll
    for (int j = 0; j < DS4_SLOTS; ++j) {
      const int e = tid + 256 * j, r = e / 100, c4 = e - 100 * r;
      if constexpr (PD) {
        const int vo = e < 1600 ? r * DRB + 8 * c4 : kOOB;
#pragma unroll
        for (int q = 0; q < 3; ++q) pv[S][j][q] = ld8(rd, vo + 2 * FG * q, 0);
      } else {
        v[S][j] = ld4(rd, e < 1600 ? (r * FG + 4 * c4) * 4 : kOOB);
      }
    }
  };
  auto stage = [&](auto S_, lds_char* buf, int j) {
    constexpr int S = decltype(S_)::value;
    const int e = tid + 256 * j, r = e / 100, c4 = e - 100 * r;
    if (e >= 1600) return;
    const int lo = (r * DS4_RS + 4 * c4) * 2;
    if constexpr (PD) {
#pragma unroll
      for (int q = 0; q < 3; ++q) *reinterpret_cast<__attribute__((address_space(3))) u32x2_t*>(buf + q * DS4_PL + lo) = pv[S][j][q];
    } else {
      uint32_t p[3][2];
      split3(v[S][j], p);
#pragma unroll
      for (int q = 0; q < 3; ++q)
        *reinterpret_cast<__attribute__((address_space(3))) u32x2_t*>(buf + q * DS4_PL + lo) = u32x2_t{p[q][0], p[q][1]};
    }
  };
  // zero the k = 400..415 pad columns of both buffers (never staged; the k-step 12 fragments read them)
  for (int i = tid; i < 2 * 3 * 16 * 2; i += 256) {
    const int h = i & 1, b = i / 96, q = (i / 32) % 3, r = (i / 2) % 16;
    *reinterpret_cast<__attribute__((address_space(3))) u32x4_t*>(dsm + b * DS4_BUF + q * DS4_PL +
                                                                  (r * DS4_RS + FG + 8 * h) * 2) = u32x4_t{0, 0, 0, 0};
  }
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  const int cs = gridDim.x;
  // prologue: this workgroup's chunk i (i = 0, 1, ...) lives in register set i % DS4_NS; chunk 0 staged
  // into buffer 0, chunks 1 .. DS4_NS - 1 in flight
  load(I0{}, blockIdx.x);
#pragma unroll
  for (int j = 0; j < DS4_SLOTS; ++j) stage(I0{}, dsm, j);
  load(I1{}, blockIdx.x + cs);
  __syncthreads();
  const int ao = (c16 * DS4_RS + 8 * g) * 2;  // this lane's A fragment: row c16, k = 8 g .. + 7 of a k-step
  // chunk cc (buffer S): chunk cc + 2 cs loaded into set S, the MFMAs on buffer S, chunk cc + cs (set
  // S ^ 1) split into buffer S ^ 1 in slices after the last DS4_SLOTS k-steps (unconditional: past
  // the end it stages zeros)
  auto chunk = [&](auto S_, int cc, int P) {  // S: register set of chunk cc, P: its LDS buffer
    constexpr int S = decltype(S_)::value, SN = (S + 1) % DS4_NS;  // SN: set of chunk cc + cs
    load(S_, cc + DS4_NS * cs);
    const lds_char* A_ = dsm + P * DS4_BUF;
    lds_char* nxt = dsm + (P ^ 1) * DS4_BUF;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    // A fragments one k-step ahead (two sets): the LDS latency hides under the previous k-step's MFMAs
    bf16x8 af[2][3];
#pragma unroll
    for (int q = 0; q < 3; ++q) af[0][q] = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(A_ + q * DS4_PL + ao);
#pragma unroll
    for (int ks = 0; ks < DS_KS; ++ks) {
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < DS_KS) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
          af[(ks + 1) & 1][q] = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(A_ + q * DS4_PL + ao + 64 * (ks + 1));
      }
      const bf16x8(&a)[3] = af[ks & 1];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        acc[e] = mma32(a[2], bw[e][ks][0], acc[e]);  // lh
        acc[e] = mma32(a[0], bw[e][ks][2], acc[e]);  // hl
        acc[e] = mma32(a[1], bw[e][ks][1], acc[e]);  // mm
        acc[e] = mma32(a[1], bw[e][ks][0], acc[e]);  // mh
        acc[e] = mma32(a[0], bw[e][ks][1], acc[e]);  // hm
        acc[e] = mma32(a[0], bw[e][ks][0], acc[e]);  // hh
      }
      if (ks >= DS4_K0) {
        stage(std::integral_constant<int, SN>{}, nxt, ks - DS4_K0);  // (compile-time)
        // in-order issue: the split's VALU only overlaps the matrix pipe when it sits BETWEEN the
        // MFMAs in program order (12 MFMAs x 16 cycles vs ~24 VALU x 4 cycles per slot)
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
      }
    }
    // output rows 16 cc + 4 g + i, columns 16 (2 w + e) + c16
    const int nr = min(16, M - 16 * cc);
    const rsrc_t rx = make_rsrc(X + (size_t)16 * cc * KO, nr * KO * 4);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int col = 16 * (2 * w + e) + c16;
      const bool ok = w < NT2 && col < KO;
#pragma unroll
      for (int i = 0; i < 4; ++i) st1(acc[e][i], rx, ok ? ((4 * g + i) * KO + col) * 4 : kOOB, 0);
    }
    __syncthreads();
  };
  int c = blockIdx.x;
  for (; c + cs < nch; c += 2 * cs) {
    chunk(I0{}, c, 0);
    chunk(I1{}, c + cs, 1);
  }
  if (c < nch) chunk(I0{}, c, 0);
}

// ==========================================================================================
// fp32 input gradient dX = dZ W^T   (dZ: M x 400, W: KO x 400 row-major, dX: M x KO, KO <= 16 NT)
// ==========================================================================================
// hipBLASLt ran this product at 59 % (KO = 100) / 41 % (KO = 32) of the fp32 MFMA pipe on the
// 6.3 M-row calls of the B = 262k step (profiles/r02_final/kernel_summary_B262144_fp32.txt,
// MT112x256x32 / MT32x256x32), 11 % of the fp32 step.
//
// One persistent workgroup per CU, 4 waves (one per SIMD), each workgroup a contiguous range of
// 16-row chunks.  Wave w owns the k-slice [100 w, 100 w + 100) of the 400-long reduction for ALL NT
// output tiles: its W^T fragments (NT x 25 k-steps) live in registers and its A operand comes
// straight from HBM into registers — every dZ byte is loaded once, by one lane, no LDS staging.
// k is permuted inside the slice (k-step 4 q + j of lane group g reads k = 16 q + 4 g + j; step 24
// reads k = 96 + g), so a lane's four consecutive k-steps are one contiguous dwordx4 (the sum over
// k is order-free; A and B use the same map).  The four waves' partial tiles meet in LDS: chunk
// c's accumulators (two alternating register sets) are written during chunk c + 1's MFMAs and
// summed in fixed wave order during chunk c + 2's, so one barrier per chunk is the only stall.
constexpr int DG_KS = 25;
template <int NT>
__global__ void __launch_bounds__(256, 1)
lstmf_dgrad_kernel(const float* __restrict__ D, const float* __restrict__ W, float* __restrict__ X, int M, int KO,
                   int rows_per_wg) {
  __shared__ __attribute__((aligned(16))) f32x4 part[2][4][NT][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int mb = blockIdx.x * rows_per_wg, nrows = min(M, mb + rows_per_wg) - mb;
  if (nrows <= 0) return;  // uniform over the workgroup
  const int kb = 100 * w;

  float bw[NT][DG_KS];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int col = 16 * n + c16;
#pragma unroll
    for (int s = 0; s < DG_KS; ++s) {
      const int k = s < 24 ? kb + 16 * (s >> 2) + 4 * g + (s & 3) : kb + 96 + g;
      bw[n][s] = col < KO ? W[col * FG + k] : 0.f;
    }
  }
  const rsrc_t rd = make_rsrc(D + (size_t)mb * FG, nrows * FG * 4);
  const rsrc_t rx = make_rsrc(X + (size_t)mb * KO, nrows * KO * 4);
  const int nch = (nrows + 15) / 16;

  f32x4 a0[6], a1[6], acc0[NT], acc1[NT];
  float s0 = 0.f, s1 = 0.f;
  auto load = [&](f32x4 (&a)[6], float& a_s, int r0) {
    const int vo = ((r0 + c16) * FG + kb + 4 * g) * 4;  // rows past the range read zeros
#pragma unroll
    for (int q = 0; q < 6; ++q) a[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, vo + 64 * q, 0, 0));
    a_s = ld1(rd, vo + (96 - 3 * g) * 4, 0);
  };
  auto mm = [&](f32x4 (&acc)[NT], const f32x4 (&a)[6], int q0, int q1) {
#pragma unroll
    for (int q = q0; q < q1; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = mma4(a[q][j], bw[n][4 * q + j], acc[n]);
  };
  auto put = [&](const f32x4 (&acc)[NT], int slot) {
#pragma unroll
    for (int n = 0; n < NT; ++n) part[slot][w][n][lane] = acc[n];
  };
  // branch-free (a fixed number of stores on every path keeps the vmcnt waits of the MFMA operand
  // loads exact); invalid lanes / chunks store to kOOB
  auto reduce = [&](int slot, int r0, bool on) {
#pragma unroll
    for (int e = 0; e < (NT * 64 + 255) / 256; ++e) {
      const int idx = tid + 256 * e, ok = on && idx < NT * 64, ix = idx < NT * 64 ? idx : 0;
      const int n = ix >> 6, ln = ix & 63, col = 16 * n + (ln & 15), row = r0 + 4 * (ln >> 4);
      const f32x4 v = ((part[slot][0][n][ln] + part[slot][1][n][ln]) + part[slot][2][n][ln]) + part[slot][3][n][ln];
#pragma unroll
      for (int i = 0; i < 4; ++i) st1(v[i], rx, ok && col < KO ? ((row + i) * KO + col) * 4 : kOOB, 0);
    }
  };
  // chunk c: chunk c - 2's partials are reduced and stored FIRST (vmcnt is in order over loads and
  // stores: stores issued after the next chunk's loads would be waited for with them), then the
  // next chunk's A operands are loaded, then the MFMAs run into cur with chunk c - 1's
  // accumulators (prev) written to LDS under them
  auto chunk = [&](f32x4 (&cur)[NT], const f32x4 (&prev)[NT], const f32x4 (&a)[6], float a_s, f32x4 (&an)[6],
                   float& an_s, int c) {
    reduce(c & 1, 16 * (c - 2), c >= 2);
    load(an, an_s, 16 * (c + 1));  // past the end: out of range, zeros
    __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMAs (the scheduler sinks them)
#pragma unroll
    for (int n = 0; n < NT; ++n) cur[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    mm(cur, a, 0, 2);
    if (c >= 1) put(prev, (c - 1) & 1);
    mm(cur, a, 2, 6);
#pragma unroll
    for (int n = 0; n < NT; ++n) cur[n] = mma4(a_s, bw[n][24], cur[n]);
    __syncthreads();
  };

  // unrolled by two so the A-operand and accumulator sets alternate without register copies
  load(a0, s0, 0);
  int c = 0;
  for (; c + 2 <= nch; c += 2) {
    chunk(acc0, acc1, a0, s0, a1, s1, c);
    chunk(acc1, acc0, a1, s1, a0, s0, c + 1);
  }
  if (c < nch) chunk(acc0, acc1, a0, s0, a1, s1, c++);
  // drain (c == nch): the last chunk's accumulators, then the last two reductions
  if (c & 1)
    put(acc0, (c - 1) & 1);
  else
    put(acc1, (c - 1) & 1);
  reduce(c & 1, 16 * (c - 2), c >= 2);
  __syncthreads();
  reduce((c - 1) & 1, 16 * (c - 1), true);
}

// ==========================================================================================
// host side
// ==========================================================================================
namespace {
constexpr size_t F_LDS_MAX = 160 * 1024;
template <int KX>
constexpr size_t fwdf_smem() {
  return (size_t)(2 * 32 * FGeo<KX>::LR + 2 * 32 * FGeo<FH>::LR + f_nwl<KX>() * 4 * FNT * 64 + 4) * 4;
}
static_assert(fwdf_smem<100>() <= F_LDS_MAX, "fp32 forward LDS");

void allow_lds(const void* k) {
  static std::mutex mu;
  static std::set<const void*> done;
  std::lock_guard<std::mutex> gd(mu);
  if (done.insert(k).second)
    HFREP_CHECK_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)F_LDS_MAX));
}
template <int KX>
constexpr size_t fwds_smem() {
  return (size_t)(2 * 32 * FGeo<KX>::LR) * 4 + 2 * FS_HB + 16;
}
// Precision modes of the fp32 path.  Default: the fp32-accurate kernels -- products of the recurrences
// (K <= 36 forwards, BPTT), both weight gradients and the K = 100 input gradient as the three-term bf16
// split (each fp32 operand = h + m + l by truncation, six of the nine products on the bf16 MFMA with
// fp32 accumulation; error <= 2x the exact kernel's vs fp64, tests/test_kernels_gpu.py).
// HFREP_FP32_EXACT=1: every product on the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32, an fmaf chain).
static bool fp32_exact() {
  return fp32_exact_mode();
}
// forward: 1 exact, 2 the split-recurrent forward for the K <= 36 layers (lstmf_fwds_kernel)
static std::atomic<int>& fwdf_impl() {
  static std::atomic<int> v{fp32_exact() ? 1 : 2};
  return v;
}
static int fwdf_version() { return fwdf_impl().load(std::memory_order_relaxed); }
template <int ACT, int KX, bool TAPE, bool TAN>
void fwdf_launch(const float* x, const float* W, const float* b, const float* U, const float* pt, float* hs, float* tp,
                 int B, int Tn, hipStream_t s) {
  const int nrb = (B + 31) / 32, cus = device_cu_count();
  // (K = 35 / 36 tangent forwards: the split kernel spills there -- registers; they stay exact)
  if constexpr (FGeo<KX>::KS <= 8 || (FGeo<KX>::KS <= 12 && !TAN)) {
    if (fwdf_version() == 2) {
      auto k = lstmf_fwds_kernel<ACT, KX, TAPE, TAN>;
      allow_lds(reinterpret_cast<const void*>(k));
      hipLaunchKernelGGL(k, dim3(nrb < cus ? nrb : cus), dim3(256), fwds_smem<KX>(), s, x, W, b, U, pt, hs, tp, B, Tn);
      return;
    }
  }
  auto k = lstmf_fwd_kernel<ACT, KX, TAPE, TAN>;
  allow_lds(reinterpret_cast<const void*>(k));
  hipLaunchKernelGGL(k, dim3(nrb < cus ? nrb : cus), dim3(256), fwdf_smem<KX>(), s, x, W, b, U, pt, hs, tp, B, Tn);
}
template <int KX, bool TAPE, bool TAN>
void fwdf_act(int act, const float* x, const float* W, const float* b, const float* U, const float* pt, float* hs,
              float* tp, int B, int Tn, hipStream_t s) {
  switch (act) {
    case ACT_LINEAR: fwdf_launch<ACT_LINEAR, KX, TAPE, TAN>(x, W, b, U, pt, hs, tp, B, Tn, s); break;
    case ACT_SIGMOID: fwdf_launch<ACT_SIGMOID, KX, TAPE, TAN>(x, W, b, U, pt, hs, tp, B, Tn, s); break;
    default: fwdf_launch<ACT_TANH, KX, TAPE, TAN>(x, W, b, U, pt, hs, tp, B, Tn, s); break;
  }
}
template <bool TAPE, bool TAN>
bool fwdf_k(int K, int act, const float* x, const float* W, const float* b, const float* U, const float* pt, float* hs,
            float* tp, int B, int Tn, hipStream_t s) {
  switch (K) {
    case 32: fwdf_act<32, TAPE, TAN>(act, x, W, b, U, pt, hs, tp, B, Tn, s); return true;
    case 35: fwdf_act<35, TAPE, TAN>(act, x, W, b, U, pt, hs, tp, B, Tn, s); return true;
    case 36: fwdf_act<36, TAPE, TAN>(act, x, W, b, U, pt, hs, tp, B, Tn, s); return true;
    case 100: fwdf_act<100, TAPE, TAN>(act, x, W, b, U, pt, hs, tp, B, Tn, s); return true;
    default: return false;
  }
}
}  // namespace

int set_lstmf_fwd_impl(int v) { return fwdf_impl().exchange(v); }

bool lstmf_supported(int H, int K, int act) {
  return H == FH && (K == 32 || K == 35 || K == 36 || K == 100) && (act == ACT_LINEAR || act == ACT_SIGMOID || act == ACT_TANH);
}

bool launch_lstmf_fwd(const float* x, const float* W, const float* b, const float* U, float* hs, float* tape, int B,
                      int Tn, int K, int H, int act, hipStream_t s) {
  if (!lstmf_supported(H, K, act) || B <= 0 || Tn <= 0) return false;
  if (tape) return fwdf_k<true, false>(K, act, x, W, b, U, nullptr, hs, tape, B, Tn, s);
  return fwdf_k<false, false>(K, act, x, W, b, U, nullptr, hs, nullptr, B, Tn, s);
}

bool launch_lstmf_tfwd(const float* xd, const float* W, const float* U, const float* tape, float* hds, float* ttape,
                       int B, int Tn, int K, int H, int act, hipStream_t s) {
  if (!lstmf_supported(H, K, act) || B <= 0 || Tn <= 0) return false;
  return fwdf_k<true, true>(K, act, xd, W, nullptr, U, tape, hds, ttape, B, Tn, s);
}

// BPTT: 2 the exact-fp32 role split (lstmf_bwdp_kernel), 3 the split-recurrent BPTT (lstmf_bwds_kernel)
static std::atomic<int>& bwdf_impl() {
  static std::atomic<int> v{fp32_exact() ? 2 : 3};
  return v;
}
template <int ACT>
void bwdf_launch(const float* dH, const float* tape, const float* U, float* dZ, int B, int Tn, hipStream_t s,
                 const float* hd, const float* hw) {
  const int ver = bwdf_impl().load(std::memory_order_relaxed);
  const int nrb = (B + 31) / 32, cus = device_cu_count();
  const size_t sm = (size_t)(32 * BZ_LR + 32 * BH_LR + 4 * BZ_KQ) * 4;
  if (ver != 2) {
    auto go = [&](auto k) {
      allow_lds(reinterpret_cast<const void*>(k));
      hipLaunchKernelGGL(k, dim3(nrb < cus ? nrb : cus), dim3(256), sm + 16 + 3 * BS_PL, s, dH, tape, U, dZ, B, Tn, hd,
                         hw);
    };
    if (hd) go(lstmf_bwds_kernel<ACT, true>);
    else go(lstmf_bwds_kernel<ACT, false>);
    return;
  }
  if (hd) throw std::runtime_error("lstmf_bwd: the exact-fp32 BPTT takes a materialised dH (lstmf_head_supported)");
  auto k = lstmf_bwdp_kernel<ACT>;
  allow_lds(reinterpret_cast<const void*>(k));
  hipLaunchKernelGGL(k, dim3(nrb < cus ? nrb : cus), dim3(512), sm, s, dH, tape, U, dZ, B, Tn);
}
static_assert((32 * BZ_LR + 32 * BH_LR + 4 * BZ_KQ) * 4 + 16 + 3 * BS_PL <= F_LDS_MAX, "split BPTT LDS");
int set_lstmf_bwd_impl(int v) { return bwdf_impl().exchange(v); }
bool lstmf_head_supported() { return bwdf_impl().load(std::memory_order_relaxed) != 2; }
bool launch_lstmf_bwd(const float* dH, const float* tape, const float* U, float* dZ, int B, int Tn, int H, int act,
                      hipStream_t s, const float* hd, const float* hw) {
  if (H != FH || B <= 0 || Tn <= 0) return false;
  switch (act) {
    case ACT_LINEAR: bwdf_launch<ACT_LINEAR>(dH, tape, U, dZ, B, Tn, s, hd, hw); return true;
    case ACT_SIGMOID: bwdf_launch<ACT_SIGMOID>(dH, tape, U, dZ, B, Tn, s, hd, hw); return true;
    case ACT_TANH: bwdf_launch<ACT_TANH>(dH, tape, U, dZ, B, Tn, s, hd, hw); return true;
    default: return false;
  }
}

template <int ACT>
void tbwdf_launch(const float* dH, const float* dHd, const float* tape, const float* ttape, const float* U, float* dZ,
                  float* dZd, int B, int Tn, hipStream_t s, const float* hd, const float* hdd, const float* hw) {
  const int cus = device_cu_count();
  const size_t sm = (size_t)(2 * 32 * BZ_LR + 2 * 32 * BH_LR + 4 * BZ_KQ) * 4;
  const int nrb = (B + 31) / 32;
  auto go = [&](auto k) {
    allow_lds(reinterpret_cast<const void*>(k));
    hipLaunchKernelGGL(k, dim3(nrb < cus ? nrb : cus), dim3(512), sm, s, dH, dHd, tape, ttape, U, dZ, dZd, B, Tn, hd, hdd,
                       hw);
  };
  if (hw) go(lstmf_tbwdp_kernel<ACT, true>);
  else go(lstmf_tbwdp_kernel<ACT, false>);
}
bool launch_lstmf_tbwd(const float* dH, const float* dHd, const float* tape, const float* ttape, const float* U, float* dZ,
                       float* dZd, int B, int Tn, int H, int act, hipStream_t s, const float* hd, const float* hdd,
                       const float* hw) {
  if (H != FH || B <= 0 || Tn <= 0) return false;
  switch (act) {
    case ACT_LINEAR: tbwdf_launch<ACT_LINEAR>(dH, dHd, tape, ttape, U, dZ, dZd, B, Tn, s, hd, hdd, hw); return true;
    case ACT_SIGMOID: tbwdf_launch<ACT_SIGMOID>(dH, dHd, tape, ttape, U, dZ, dZd, B, Tn, s, hd, hdd, hw); return true;
    case ACT_TANH: tbwdf_launch<ACT_TANH>(dH, dHd, tape, ttape, U, dZ, dZd, B, Tn, s, hd, hdd, hw); return true;
    default: return false;
  }
}
size_t lstmf_tape_elems(int B, int Tn) { return (size_t)((B + 31) / 32) * Tn * FT_STEP; }

static int wgradf_grid(int M) {
  const int chunks = (M + WF_R - 1) / WF_R, cus = device_cu_count();
  return chunks < cus ? chunks : cus;
}
bool lstmf_wgrad_supported(int K, int H, int N) { return H == FH && N == FG && (K == 32 || K == 35 || K == 36 || K == 100); }

// impl 1 / 2 / 3: the exact-fp32 MFMA kernel / the three-term bf16 split (pair) / the split quad;
// default (0): exact under HFREP_FP32_EXACT, else the pair split for K <= 36 (12.1 -> 9.8 ms at 12.6 M
// rows), the quad for K = 100 (16.4 -> 15.3 ms; the pair kernel's 28-tile waves spill there: 52.8 ms;
// profiles/r03_split)
static int wgradf_version() { return fp32_exact() ? 1 : 0; }
// split kernel: Z row ranges x 2 column halves, one workgroup per CU
static int wgrads_z(int M) {
  const int chunks = (M + 31) / 32, half = device_cu_count() / 2;
  return chunks < half ? chunks : half;
}
// quad kernel: Z row ranges x 4 column quarters, one workgroup per CU
static int wgradq_z(int M) {
  const int chunks = (M + 31) / 32, q = device_cu_count() / 4;
  return chunks < q ? chunks : q;
}
static int wgradf_pick(int impl, int K, int M) {
  (void)M;
  int v = impl >= 1 && impl <= 3 ? impl : wgradf_version();
  if (K == 35 && v == 3) v = 2;  // the quad kernel reads 16-byte X rows only
  return v ? v : (K <= 36 ? 2 : 3);
}
size_t lstmf_wgrad_workspace_floats(int M, int K, int impl) {
  const int v = wgradf_pick(impl, K, M);
  const int z = v == 1 ? wgradf_grid(M) : v == 3 ? wgradq_z(M) : wgrads_z(M);
  return (size_t)z * ((K == 35 ? 36 : K) + FH + 1) * FG;
}

bool launch_lstmf_wgrad(const void* X, const void* Hs, const void* D, const void* Xd, const void* Hds, const void* Dd,
                        float* gW, float* gU, float* gb, int M, int K, int Tn, float* ws, hipStream_t s, int impl, int pm) {
  if (!lstmf_wgrad_supported(K, FH, FG) || M <= 0) return false;
  if (pm != 0 && (wgradf_pick(impl, K, M) == 1 || K == 35 || K == 36))
    throw std::runtime_error("lstmf_wgrad: FP3-plane operands need the split kernels and K in {32, 100}");
  if (wgradf_pick(impl, K, M) == 3) {
    const int z0 = wgradq_z(M);
    const int rpz = ((M + z0 - 1) / z0 + 31) / 32 * 32;
    const int z = (M + rpz - 1) / rpz;
    auto go = [&](auto k, size_t sm) {
      allow_lds(reinterpret_cast<const void*>(k));
      hipLaunchKernelGGL(k, dim3(4 * z), dim3(512), sm, s, X, Hs, D, Xd, Hds, Dd, ws, M, Tn, rpz, z);
    };
    switch (K * 8 + pm) {
#define HFREP_Q4(KK, PP) case KK * 8 + PP: go(lstmf_wgrad_q4_kernel<KK, PP>, 2 * WQGeo<KK>::Img::BUF); break;
      HFREP_Q4(32, 0) HFREP_Q4(36, 0) HFREP_Q4(100, 0)
      HFREP_Q4(32, 4) HFREP_Q4(32, 6) HFREP_Q4(32, 7) HFREP_Q4(100, 4) HFREP_Q4(100, 6) HFREP_Q4(100, 7)
#undef HFREP_Q4
      default: throw std::runtime_error("lstmf_wgrad: no quad kernel for this K / plane mask");
    }
    launch_lstm_wgrad2_reduce(ws, gW, gU, gb, z, K, FH, FG, s);
    return true;
  }
  if (wgradf_pick(impl, K, M) != 1) {
    const int z0 = wgrads_z(M);
    const int rpz = ((M + z0 - 1) / z0 + 31) / 32 * 32;
    const int z = (M + rpz - 1) / rpz;
    auto go = [&](auto k, size_t sm) {
      allow_lds(reinterpret_cast<const void*>(k));
      hipLaunchKernelGGL(k, dim3(2 * z), dim3(512), sm, s, X, Hs, D, Xd, Hds, Dd, ws, M, Tn, rpz, z);
    };
    switch (K * 8 + pm) {
      case 35 * 8: go(lstmf_wgrad_split_kernel<36, 35>, 2 * WSGeo<36>::Img::BUF); break;
      case 36 * 8: go(lstmf_wgrad_split_kernel<36>, 2 * WSGeo<36>::Img::BUF); break;
      case 100 * 8: go(lstmf_wgrad_split_kernel<100>, 2 * WSGeo<100>::Img::BUF); break;
#define HFREP_WS(PP) case 32 * 8 + PP: go(lstmf_wgrad_split_kernel<32, 32, PP>, 2 * WSGeo<32>::Img::BUF); break;
      HFREP_WS(0) HFREP_WS(4) HFREP_WS(6) HFREP_WS(7)
#undef HFREP_WS
      default: throw std::runtime_error("lstmf_wgrad: no pair kernel for this K / plane mask");
    }
    launch_lstm_wgrad2_reduce(ws, gW, gU, gb, z, K, FH, FG, s, K == 35 ? 36 : K);
    return true;
  }
  const int grid = wgradf_grid(M);
  const int rpw = ((M + grid - 1) / grid + WF_R - 1) / WF_R * WF_R;
  const int z = (M + rpw - 1) / rpw;
  const float *Xf = static_cast<const float*>(X), *Hf = static_cast<const float*>(Hs), *Df = static_cast<const float*>(D);
  const float *Xdf = static_cast<const float*>(Xd), *Hdf = static_cast<const float*>(Hds), *Ddf = static_cast<const float*>(Dd);
  switch (K) {
    case 32: hipLaunchKernelGGL(lstmf_wgrad_kernel<32>, dim3(z), dim3(512), 0, s, Xf, Hf, Df, Xdf, Hdf, Ddf, ws, M, Tn, rpw); break;
    case 35: hipLaunchKernelGGL((lstmf_wgrad_kernel<36, 35>), dim3(z), dim3(512), 0, s, Xf, Hf, Df, Xdf, Hdf, Ddf, ws, M, Tn, rpw); break;
    case 36: hipLaunchKernelGGL(lstmf_wgrad_kernel<36>, dim3(z), dim3(512), 0, s, Xf, Hf, Df, Xdf, Hdf, Ddf, ws, M, Tn, rpw); break;
    default: hipLaunchKernelGGL(lstmf_wgrad_kernel<100>, dim3(z), dim3(512), 0, s, Xf, Hf, Df, Xdf, Hdf, Ddf, ws, M, Tn, rpw); break;
  }
  launch_lstm_wgrad2_reduce(ws, gW, gU, gb, z, K, FH, FG, s, K == 35 ? 36 : K);
  return true;
}

bool lstmf_dgrad_supported(int N, int KO) { return N == FG && KO >= 1 && KO <= 16 * FNT; }

void launch_fp3_split(const float* x, uint16_t* p, int64_t M, int C, bool interleave, hipStream_t s) {
  if (M <= 0) return;
  if (C % 4 != 0 || (interleave && C != FG)) throw std::runtime_error("fp3_split: C % 4 == 0 (400 when interleaved)");
  const int64_t n4 = M * (C / 4);
  const int grid = (int)std::min<int64_t>((n4 + 255) / 256, (int64_t)device_cu_count() * 16);
  if (interleave) hipLaunchKernelGGL(fp3_split_kernel<true>, dim3(grid), dim3(256), 0, s, x, p, M, C);
  else hipLaunchKernelGGL(fp3_split_kernel<false>, dim3(grid), dim3(256), 0, s, x, p, M, C);
}
void launch_fp3_join(const uint16_t* p, float* x, int64_t M, int C, bool interleave, hipStream_t s) {
  if (M <= 0) return;
  if (interleave && C != FG) throw std::runtime_error("fp3_join: interleaved planes are 400 wide");
  const int64_t n = M * C;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, (int64_t)device_cu_count() * 16);
  if (interleave) hipLaunchKernelGGL(fp3_join_kernel<true>, dim3(grid), dim3(256), 0, s, p, x, M, C);
  else hipLaunchKernelGGL(fp3_join_kernel<false>, dim3(grid), dim3(256), 0, s, p, x, M, C);
}

// impl 1 / 3: the exact-fp32 MFMA kernel / the LDS-staged split kernel lstmf_dgrad_s4_kernel; default
// (0): exact under HFREP_FP32_EXACT, else s4 for KO > 64 and exact otherwise (s4 keeps one wave busy
// per 32 output columns, so KO = 32 leaves three SIMDs idle; profiles/r03_split)
static int dgradf_version() { return fp32_exact() ? 1 : 0; }

bool launch_lstmf_dgrad(const void* D, const float* W, float* X, int M, int N, int KO, hipStream_t s, int impl, bool pd) {
  if (!lstmf_dgrad_supported(N, KO) || M <= 0) return false;
  const int dv = impl == 1 || impl == 3 ? impl : dgradf_version();
  if (pd && dv == 1) throw std::runtime_error("lstmf_dgrad: FP3-plane dZ needs the split kernel");
  if (pd || dv == 3 || (dv == 0 && KO > 64)) {
    const int chunks = (M + 15) / 16, cus = device_cu_count();
    const int grid = chunks < cus ? chunks : cus;
    auto go = [&](auto k) {
      allow_lds(reinterpret_cast<const void*>(k));
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), (size_t)2 * DS4_BUF, s, D, W, X, M, KO);
    };
    switch ((KO + 31) / 32 + (pd ? 4 : 0)) {
      case 1: go(lstmf_dgrad_s4_kernel<1>); break;
      case 2: go(lstmf_dgrad_s4_kernel<2>); break;
      case 3: go(lstmf_dgrad_s4_kernel<3>); break;
      case 4: go(lstmf_dgrad_s4_kernel<4>); break;
      case 5: go(lstmf_dgrad_s4_kernel<1, true>); break;
      case 6: go(lstmf_dgrad_s4_kernel<2, true>); break;
      case 7: go(lstmf_dgrad_s4_kernel<3, true>); break;
      default: go(lstmf_dgrad_s4_kernel<4, true>); break;
    }
    return true;
  }
  const float* Df = static_cast<const float*>(D);
  // one workgroup per CU (two for NT <= 3: HBM-bound there, and the registers allow a second one
  // in flight); more only if a workgroup's dZ range would pass 2 GB (32-bit buffer offsets)
  const int chunks = (M + 15) / 16, cus = device_cu_count() * (KO <= 48 ? 2 : 1);
  int grid = chunks < cus ? chunks : cus;
  const int min_grid = (int)(((long long)M * FG * 4 + (1ll << 31) - 1) / (1ll << 31));
  if (grid < min_grid) grid = min_grid;
  const int rpw = (chunks + grid - 1) / grid * 16;
  const int z = (M + rpw - 1) / rpw;
  switch ((KO + 15) / 16) {
    case 1: hipLaunchKernelGGL(lstmf_dgrad_kernel<1>, dim3(z), dim3(256), 0, s, Df, W, X, M, KO, rpw); break;
    case 2: hipLaunchKernelGGL(lstmf_dgrad_kernel<2>, dim3(z), dim3(256), 0, s, Df, W, X, M, KO, rpw); break;
    case 3: hipLaunchKernelGGL(lstmf_dgrad_kernel<3>, dim3(z), dim3(256), 0, s, Df, W, X, M, KO, rpw); break;
    case 4: hipLaunchKernelGGL(lstmf_dgrad_kernel<4>, dim3(z), dim3(256), 0, s, Df, W, X, M, KO, rpw); break;
    case 5: hipLaunchKernelGGL(lstmf_dgrad_kernel<5>, dim3(z), dim3(256), 0, s, Df, W, X, M, KO, rpw); break;
    case 6: hipLaunchKernelGGL(lstmf_dgrad_kernel<6>, dim3(z), dim3(256), 0, s, Df, W, X, M, KO, rpw); break;
    default: hipLaunchKernelGGL(lstmf_dgrad_kernel<7>, dim3(z), dim3(256), 0, s, Df, W, X, M, KO, rpw); break;
  }
  return true;
}

}  // namespace hfrep
