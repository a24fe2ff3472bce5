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

#include <mutex>
#include <set>

namespace hfrep {

namespace {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
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

}  // namespace

// ==========================================================================================
// forward / tangent forward
// ==========================================================================================
template <int ACT, int KX, bool TAPE, bool TAN>
__global__ void __launch_bounds__(256, 1)
lstmf_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                 const float* __restrict__ U, const float* __restrict__ pgates, const float* __restrict__ pcs,
                 float* __restrict__ hs, float* __restrict__ gout, float* __restrict__ cout, int B, int Tn) {
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
    const rsrc_t rgo = ftile_rsrc(gout, row0, B, Tn, FG);
    const rsrc_t rco = ftile_rsrc(cout, row0, B, Tn, FH);
    const rsrc_t rpg = ftile_rsrc(TAN ? pgates : nullptr, row0, B, Tn, FG);
    const rsrc_t rpc = ftile_rsrc(TAN ? pcs : nullptr, row0, B, Tn, FH);
    // byte offsets at step 0 of this lane's rows (the descriptors cover rows < B only, so a row
    // past B is out of range by itself): post-transpose (row 16 m + 4 g + q, unit ub) of (B,T,H) and
    // (B,T,4H); pre-transpose row 16 m + 4 g at column q H + ub of (B,T,4H).  Every store / load
    // offset below is (this base + t * row stride) + an immediate, so nothing per tile is hoisted
    // out of the step loop into registers.
    int vp1[2], vp4[2], vq4[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int r = 16 * m + 4 * g + q, r0 = 16 * m + 4 * g;
      vp1[m] = (r * Tn * FH + ub) * 4;
      vp4[m] = (r * Tn * FG + ub) * 4;
      vq4[m] = (r0 * Tn * FG + q * FH + ub) * 4;
    }
    const int rs4 = Tn * FG * 4;  // row stride of (B,T,4H)
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
        // tangent: primal gates of this lane's 4 accumulator rows, c_t and c_{t-1} of its (row, unit);
        // issued before this half's MFMAs, consumed after them
        float py[TAN ? FNT : 1][4], pc0[TAN ? FNT : 1], pc1[TAN ? FNT : 1];
        const int p1 = vp1[m] + t * FH * 4, p4 = vp4[m] + t * FG * 4, q4 = vq4[m] + t * FG * 4;
        if constexpr (TAN) {
#pragma unroll
          for (int n = 0; n < FNT; ++n) {
            const bool tok = !(w == 3 && n >= 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) py[n][i] = ld1(rpg, tok ? q4 + i * rs4 + 16 * n : kOOB, 0);
            pc0[n] = ld1(rpc, tok ? p1 + 16 * n : kOOB, 0);
            pc1[n] = ld1(rpc, (tok && t > 0) ? p1 - FH * 4 + 16 * n : kOOB, 0);
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
              const int v4 = tok ? p4 + 16 * n : kOOB;
#pragma unroll
              for (int k = 0; k < 4; ++k) st1(y[k], rgo, v4 + k * FH * 4, 0);
              st1(cn, rco, v1, 0);
            }
          } else {
            float gd[4], y[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float yy = py[n][i];
              const float der = q == 2 ? act_dy(ACT, yy) : yy * (1.f - yy);
              gd[i] = der * acc[n][i];
              y[i] = yy;
              // zdot, pre-transpose: row 16 m + 4 g + i, gate q, unit ub + 4 n
              st1(acc[n][i], rgo, tok ? q4 + i * rs4 + 16 * n : kOOB, 0);
            }
            quad_transpose(gd, q);
            quad_transpose(y, q);
            const float c = pc0[n], cp = pc1[n];
            float cdn = gd[1] * cp + y[1] * cst[m][n] + gd[0] * y[2] + y[0] * gd[2];
            const float ca = act_f(ACT, c);
            float hd = gd[3] * ca + y[3] * act_dy(ACT, ca) * cdn;
            if (!tok) { cdn = 0.f; hd = 0.f; }
            cst[m][n] = cdn;
            hv = hd;
            st1(cdn, rco, v1, 0);
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

template <int KX>
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
    const rsrc_t rx = make_rsrc(Xs, M * KX * 4), rh = make_rsrc(Hq, M * FH * 4), rd = make_rsrc(Dq, M * FG * 4);
    auto load = [&](int m0) {
#pragma unroll
      for (int j = 0; j < WG::JX; ++j) {
        const int e = tid + 512 * j, r = e / (KX / 4), c = e - r * (KX / 4);
        const bool ok = e < WG::NX4 && m0 + r < me;
        vx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? ((m0 + r) * KX + 4 * c) * 4 : kOOB, 0, 0));
      }
#pragma unroll
      for (int j = 0; j < WG::JH; ++j) {
        const int e = tid + 512 * j, r = e / (FH / 4), c = e - r * (FH / 4);
        const int m = m0 + r;
        const bool ok = e < WG::NH4 && m < me && (m % Tn) != 0;  // h_{-1} = 0 at t = 0
        vh[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, ok ? ((m - 1) * FH + 4 * c) * 4 : kOOB, 0, 0));
      }
#pragma unroll
      for (int j = 0; j < WG::JD; ++j) {
        const int e = tid + 512 * j, r = e / (FG / 4), c = e - r * (FG / 4);
        const bool ok = e < WG::ND4 && m0 + r < me;
        vd[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, ok ? ((m0 + r) * FG + 4 * c) * 4 : kOOB, 0, 0));
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
template <int ACT, int KX, bool TAPE, bool TAN>
void fwdf_launch(const float* x, const float* W, const float* b, const float* U, const float* pg, const float* pc, float* hs,
                 float* go, float* co, int B, int Tn, hipStream_t s) {
  auto k = lstmf_fwd_kernel<ACT, KX, TAPE, TAN>;
  allow_lds(reinterpret_cast<const void*>(k));
  const int nrb = (B + 31) / 32, cus = device_cu_count();
  hipLaunchKernelGGL(k, dim3(nrb < cus ? nrb : cus), dim3(256), fwdf_smem<KX>(), s, x, W, b, U, pg, pc, hs, go, co, B, Tn);
}
template <int KX, bool TAPE, bool TAN>
void fwdf_act(int act, const float* x, const float* W, const float* b, const float* U, const float* pg, const float* pc,
              float* hs, float* go, float* co, int B, int Tn, hipStream_t s) {
  switch (act) {
    case ACT_LINEAR: fwdf_launch<ACT_LINEAR, KX, TAPE, TAN>(x, W, b, U, pg, pc, hs, go, co, B, Tn, s); break;
    case ACT_SIGMOID: fwdf_launch<ACT_SIGMOID, KX, TAPE, TAN>(x, W, b, U, pg, pc, hs, go, co, B, Tn, s); break;
    default: fwdf_launch<ACT_TANH, KX, TAPE, TAN>(x, W, b, U, pg, pc, hs, go, co, B, Tn, s); break;
  }
}
template <bool TAPE, bool TAN>
bool fwdf_k(int K, int act, const float* x, const float* W, const float* b, const float* U, const float* pg,
            const float* pc, float* hs, float* go, float* co, int B, int Tn, hipStream_t s) {
  switch (K) {
    case 32: fwdf_act<32, TAPE, TAN>(act, x, W, b, U, pg, pc, hs, go, co, B, Tn, s); return true;
    case 35: fwdf_act<35, TAPE, TAN>(act, x, W, b, U, pg, pc, hs, go, co, B, Tn, s); return true;
    case 36: fwdf_act<36, TAPE, TAN>(act, x, W, b, U, pg, pc, hs, go, co, B, Tn, s); return true;
    case 100: fwdf_act<100, TAPE, TAN>(act, x, W, b, U, pg, pc, hs, go, co, B, Tn, s); return true;
    default: return false;
  }
}
}  // namespace

bool lstmf_supported(int H, int K, int act) {
  return H == FH && (K == 32 || K == 35 || K == 36 || K == 100) && (act == ACT_LINEAR || act == ACT_SIGMOID || act == ACT_TANH);
}

bool launch_lstmf_fwd(const float* x, const float* W, const float* b, const float* U, float* hs, float* gates, float* cs,
                      int B, int Tn, int K, int H, int act, hipStream_t s) {
  if (!lstmf_supported(H, K, act) || B <= 0 || Tn <= 0) return false;
  if (gates) return fwdf_k<true, false>(K, act, x, W, b, U, nullptr, nullptr, hs, gates, cs, B, Tn, s);
  return fwdf_k<false, false>(K, act, x, W, b, U, nullptr, nullptr, hs, nullptr, nullptr, B, Tn, s);
}

bool launch_lstmf_tfwd(const float* xd, const float* W, const float* U, const float* gates, const float* cs, float* hds,
                       float* zds, float* cds, int B, int Tn, int K, int H, int act, hipStream_t s) {
  if (!lstmf_supported(H, K, act) || B <= 0 || Tn <= 0) return false;
  return fwdf_k<true, true>(K, act, xd, W, nullptr, U, gates, cs, hds, zds, cds, B, Tn, s);
}

static int wgradf_grid(int M) {
  const int chunks = (M + WF_R - 1) / WF_R, cus = device_cu_count();
  return chunks < cus ? chunks : cus;
}
bool lstmf_wgrad_supported(int K, int H, int N) { return H == FH && N == FG && (K == 32 || K == 36 || K == 100); }
size_t lstmf_wgrad_workspace_floats(int M, int K) { return (size_t)wgradf_grid(M) * (K + FH + 1) * FG; }

bool launch_lstmf_wgrad(const float* X, const float* Hs, const float* D, const float* Xd, const float* Hds, const float* Dd,
                        float* gW, float* gU, float* gb, int M, int K, int Tn, float* ws, hipStream_t s) {
  if (!lstmf_wgrad_supported(K, FH, FG) || M <= 0) return false;
  const int grid = wgradf_grid(M);
  const int rpw = ((M + grid - 1) / grid + WF_R - 1) / WF_R * WF_R;
  const int z = (M + rpw - 1) / rpw;
  switch (K) {
    case 32: hipLaunchKernelGGL(lstmf_wgrad_kernel<32>, dim3(z), dim3(512), 0, s, X, Hs, D, Xd, Hds, Dd, ws, M, Tn, rpw); break;
    case 36: hipLaunchKernelGGL(lstmf_wgrad_kernel<36>, dim3(z), dim3(512), 0, s, X, Hs, D, Xd, Hds, Dd, ws, M, Tn, rpw); break;
    default: hipLaunchKernelGGL(lstmf_wgrad_kernel<100>, dim3(z), dim3(512), 0, s, X, Hs, D, Xd, Hds, Dd, ws, M, Tn, rpw); break;
  }
  launch_lstm_wgrad2_reduce(ws, gW, gU, gb, z, K, FH, FG, s);
  return true;
}

}  // namespace hfrep
