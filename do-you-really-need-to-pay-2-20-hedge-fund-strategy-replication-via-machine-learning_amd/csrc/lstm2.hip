// LSTM layer kernels v2 (bf16, gfx950): fused input projection + blocked tapes.
//
// v1 (lstm.hip) consumed a materialised zx = x W + b (B,T,4H) and saved gate activations in the
// row-major (B,T,4H) layout, which the 32x32 accumulator layout can only touch with 2-byte,
// lane-scattered global accesses (profiles/r01_baseline: ~0.7 TB/s, 28 TF/s).  v2:
//
//  * the input projection runs inside the recurrence: W^T (4H x K) is staged once per workgroup
//    in LDS (bf16) and z_t = x_t W + h_{t-1} U + b is ONE MFMA chain per gate; x_t tiles are
//    prefetched one step ahead into registers and written to a double-buffered LDS tile, so the
//    HBM latency hides under the previous step's MFMA + gate math.  zx never exists in HBM;
//  * tapes (gate activations + cell state for BPTT; tangent pre-activations + cell tangent for the
//    GP's reverse pass) are stored in a BLOCKED layout [rowblock][t][wave][slot][half][lane][8]
//    that matches the accumulator layout: each lane moves its 16 values with two 16-byte accesses
//    and every wave-level access covers 1 KiB of contiguous memory;
//  * row-major activations (h, dH, dZ) go through the LDS tile that the recurrence needs anyway
//    and are streamed to/from HBM with coalesced 8-byte accesses by the whole workgroup.
//
// Contracts are identical to ops/reference.py (lstm_seq_*), with zx = x W + b folded in.
//
// File map:
//   buffer descriptors, tile movers, tape slot I/O ........ shared device helpers
//   lstm_tfwd2 .............................................. v2 tangent forward (32x32x16, 32 units per
//                                                            wave): dispatched for act = sigmoid only
//   lstm_tbwd4 .............................................. tangent reverse: 16x16x32, 7 + 1 waves;
//                                                            TG = false: the BPTT
//   lstm_fwd4 ............................................... forward + tangent forward: 16x16x32
//   host side ............................................... launchers
// Every v3 / v4 kernel: one persistent workgroup per CU walking 32-row tiles, 2 waves per SIMD
// (<= 256 VGPRs, no spills), row-major tiles moved HBM <-> LDS by the data waves, tapes in the
// blocked 32x32-accumulator layout, buffer-descriptor (range-checked) global accesses.
#include "common.h"
#include "mfma.h"
#include "kernels.h"

#include <cstdlib>
#include <mutex>
#include <set>

namespace hfrep {

namespace {

constexpr int NW2 = 4;       // waves per workgroup: 4 x 32 units covers H <= 128
constexpr int TAPE_SLOTS = 5;  // 4 gates (or 4 tangent pre-activations) + cell (or cell tangent)
constexpr int SLOT_ELEMS = 64 * 16;
// a slot is [half][lane][8]: lane l's 16 values are two 16-byte pieces 1 KiB apart, so every
// wave-level 16-byte store / load of a tape slot covers one contiguous 1 KiB (whole cache lines;
// the [lane][16] form left 16-byte holes in every line and cost ~1/3 of lstm_fwd2's time)
constexpr int SLOT_HALF = 64 * 8;

__device__ __forceinline__ size_t tape_base(int rb, int t, int Tn, int w) {
  return (((size_t)rb * Tn + t) * NW2 + w) * TAPE_SLOTS * SLOT_ELEMS;
}
// element offset of (t, wave w) inside one row block's tape region
__device__ __forceinline__ int tape_off(int t, int w) { return (t * NW2 + w) * TAPE_SLOTS * SLOT_ELEMS; }

// ---------------------------------------------------------------------------------------------
// Buffer descriptors.  Every global access of the step loops goes through a buffer resource
// (SRD) that covers one 32-row tile (or one row block's tape region) and nothing else: rows past
// B, padded unit lanes, idle trailing tiles and the out-of-range neighbours of the first / last
// step get an offset beyond num_records, so the hardware range check turns their loads into
// zeros and drops their stores.  Each thread therefore issues the SAME memory instructions in
// every step, without exec-masked branches, and that matters on CDNA4: vmcnt retires loads and
// stores together in issue order, and a wait the compiler computes across a branch that may skip
// some stores must assume the shortest path, i.e. wait for stores it never needed (the waits in
// the v2 step loops were vmcnt(0) behind the step's own tile stores; profiles/r01_vmcnt).
// The range check looks at voffset only (soffset is added to the base address unchecked): the row
// of an access always lives in voffset, and soffset carries only step / wave / slot offsets that
// are in range whenever the voffset part is.  Per-lane parts in voffset, uniform parts in soffset
// also keeps the loop-invariant address registers to one or two per access group.
// ---------------------------------------------------------------------------------------------
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kOOB = 0x7fff0000;  // byte offset past every descriptor's num_records

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
// rows [row0, min(row0 + 32, B)) of a row-major (B, Tn, W) bf16 tensor; a null base or a tile
// past B gets zero records
__device__ __forceinline__ rsrc_t tile_rsrc(const bf16_t* base, int row0, int B, int Tn, int W) {
  row0 = __builtin_amdgcn_readfirstlane(row0);
  const int nr = base ? max(0, min(32, B - row0)) : 0;
  return make_rsrc(base + (nr ? (size_t)row0 * Tn * W : 0), nr * Tn * W * 2);
}
// one row block's tape region ([t][wave][slot][half][lane][8])
__device__ __forceinline__ rsrc_t tape_rsrc(const bf16_t* tape, int rb, int nrb, int Tn) {
  rb = __builtin_amdgcn_readfirstlane(rb);
  const bool on = tape && rb < nrb;
  return make_rsrc(tape + (on ? tape_base(rb, 0, Tn, 0) : 0), on ? Tn * NW2 * TAPE_SLOTS * SLOT_ELEMS * 2 : 0);
}

__device__ __forceinline__ uint32_t pk2(float lo, float hi) { return pk2bf(lo, hi); }
__device__ __forceinline__ float lo_bf(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float hi_bf(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }

struct Slot16 {  // 16 bf16 values of one lane, packed
  uint4 a, b;
  __device__ __forceinline__ float get(int r) const {
    const uint32_t w = (r < 8) ? ((r >> 1) == 0 ? a.x : (r >> 1) == 1 ? a.y : (r >> 1) == 2 ? a.z : a.w)
                               : (((r - 8) >> 1) == 0 ? b.x : ((r - 8) >> 1) == 1 ? b.y : ((r - 8) >> 1) == 2 ? b.z : b.w);
    return (r & 1) ? hi_bf(w) : lo_bf(w);
  }
};
// lanes whose unit is padding (u >= H: 28 of 128 tape columns) neither load nor store (their
// offsets are out of range): the tape's padded slots are never touched, which trims 22% of the
// tape traffic.  `off` is this lane's element offset of the slot's first half.
__device__ __forceinline__ Slot16 ld_slot(rsrc_t rs, bool on, int lane_off, int uoff) {
  Slot16 s;
  const int v = on ? lane_off * 2 : kOOB;
  s.a = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, v, uoff * 2, 0));
  s.b = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, v, (uoff + SLOT_HALF) * 2, 0));
  return s;
}
// 16-byte STORES keep soffset = 0: a buffer store of more than 8 bytes whose data VGPRs a VALU
// instruction overwrites right after it needs one wait state, and the compiler's hazard model
// omits it when soffset is a register (measured on gfx950: the 4th tape slot came back corrupt)
__device__ __forceinline__ void st_slot(rsrc_t rs, bool on, int lane_off, int uoff, const uint32_t (&v)[4]) {
  const v4i d = {(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
  __builtin_amdgcn_raw_buffer_store_b128(d, rs, on ? (lane_off + uoff) * 2 : kOOB, 0, 0);
}
__device__ __forceinline__ void put4(uint32_t (&v)[4], int i, float x) {
  if (i & 1) v[i >> 1] |= ((uint32_t)f2bf(x) << 16);
  else v[i >> 1] = (uint32_t)f2bf(x);
}

// stage W^T (K x G fp32, row-major) into LDS as bf16 [G][LX], zero-padded in k
__device__ __forceinline__ void stage_wt(bf16_t* Wt, const float* __restrict__ W, int K, int G, int LX) {
#pragma unroll 4
  for (int e = threadIdx.x; e < G * LX; e += blockDim.x) {
    const int k = e / G, n = e % G;  // consecutive threads read consecutive n (coalesced)
    const float v = W[(size_t)min(k, K - 1) * G + n];  // in-bounds load, then select: no per-element branch
    Wt[n * LX + k] = f2bf(k < K ? v : 0.f);
  }
}

// x tile (32 rows x K, time t) -> registers.  KX > 0 (K % 4 == 0, the model's widths) makes K and
// every index division a compile-time constant and moves 8-byte chunks (XJ per thread of the tile's
// 256 threads); KX == 0 is the generic path for any K <= 128 (one element at a time, 16 per thread).
template <int KX>
struct XGeo {
  static constexpr bool VEC = KX > 0 && KX % 4 == 0;  // 8-byte chunks; else one element at a time
  static constexpr int XJ = VEC ? (32 * KX / 4 + 255) / 256 : 4;
  static_assert(XJ <= 4, "x tile");
};
struct XPref {
  uint2 v[4];
};
// x tile of step t through the tile descriptor `rx` (rows past B read 0); `on` == false (a step
// outside [0, Tn)) issues the same loads out of range
template <int KX>
__device__ __forceinline__ void x_load(XPref& p, rsrc_t rx, int Tn, int t, bool on, int K, int ltid) {
  if constexpr (!XGeo<KX>::VEC) {
    if constexpr (KX > 0) K = KX;
    uint32_t* pv = reinterpret_cast<uint32_t*>(p.v);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int e = ltid + 256 * j;
      const int r = e / K, k = e - r * K;
      const int off = (on && r < 32) ? (r * Tn * K + k) * 2 : kOOB;  // step t in soffset
      const uint32_t v = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rx, off, t * K * 2, 0);
      if (j & 1) pv[j >> 1] |= v << 16;
      else pv[j >> 1] = v;
    }
  } else {
    constexpr int K4 = KX / 4;
#pragma unroll
    for (int j = 0; j < XGeo<KX>::XJ; ++j) {
      const int e = ltid + 256 * j;
      const int r = e / K4, c = e - r * K4;
      const int off = (on && r < 32) ? (r * Tn * KX + 4 * c) * 2 : kOOB;  // step t in soffset
      p.v[j] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rx, off, t * KX * 2, 0));
    }
  }
}
template <int KX>
__device__ __forceinline__ void x_store_lds(const XPref& p, bf16_t* xb, int K, int LX, int ltid) {
  if constexpr (!XGeo<KX>::VEC) {
    if constexpr (KX > 0) K = KX;
    const uint32_t* pv = reinterpret_cast<const uint32_t*>(p.v);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int e = ltid + 256 * j;
      const int r = e / K, k = e - r * K;
      if (r < 32) xb[r * LX + k] = (bf16_t)((j & 1) ? (pv[j >> 1] >> 16) : (pv[j >> 1] & 0xffffu));
    }
  } else {
    constexpr int K4 = KX / 4;
#pragma unroll
    for (int j = 0; j < XGeo<KX>::XJ; ++j) {
      const int e = ltid + 256 * j;
      const int r = e / K4, c = e - r * K4;
      if (r < 32) *reinterpret_cast<uint2*>(xb + r * LX + 4 * c) = p.v[j];
    }
  }
}

// Source of the dH (dHdot) tiles of the reverse kernels, moved by NT threads in 8-byte chunks:
// GEN = false: a row-major (B, T, W) tensor (`rs` = its tile descriptor);
// GEN = true: the outer product d[b] * w[t W + h] of a Flatten -> Dense(1) critic head, generated
// in-kernel (`rs` = descriptor over the tile's rows of d (B, 1), `rw` over w (T W floats)), so the
// head's (B, T, W) input adjoint is never written to HBM nor read back.  The product is rounded
// exactly as the skinny dgrad kernel rounds it (bf16(float(d) * w)).
template <int W, int NT, bool GEN>
struct TileSrc {
  static constexpr int CPR = W / 4, NJ = (32 * CPR + NT - 1) / NT;
  static_assert(W % 4 == 0, "8-byte chunks");
  v2i v[GEN ? 1 : NJ];
  uint32_t d[GEN ? NJ : 1];
  float4 wv[GEN ? NJ : 1];
  __device__ __forceinline__ void load(rsrc_t rs, rsrc_t rw, int Tn, int t, bool on, int tid) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int e = tid + NT * j;
      const int r = e / CPR, c = e - r * CPR;
      const bool ok = on && r < 32;
      if constexpr (!GEN) {
        v[j] = __builtin_amdgcn_raw_buffer_load_b64(rs, ok ? (r * Tn * W + 4 * c) * 2 : kOOB, t * W * 2, 0);
      } else {
        d[j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, ok ? r * 2 : kOOB, 0, 0);
        wv[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? (t * W + 4 * c) * 4 : kOOB, 0, 0));
      }
    }
  }
  __device__ __forceinline__ void to_lds(bf16_t* buf, int LD, int tid) const {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int e = tid + NT * j;
      const int r = e / CPR, c = e - r * CPR;
      if (r < 32) {
        v2i o;
        if constexpr (!GEN) {
          o = v[j];
        } else {
          const float dv = __uint_as_float(d[j] << 16);
          o = v2i{(int)pk2(dv * wv[j].x, dv * wv[j].y), (int)pk2(dv * wv[j].z, dv * wv[j].w)};
        }
        *reinterpret_cast<v2i*>(buf + r * LD + 4 * c) = o;
      }
    }
  }
};
// tile descriptors of a dH source: (tensor tile, unused) or (rows of d, all of w)
template <int W, bool GEN>
__device__ __forceinline__ void head_rsrc(rsrc_t& rs, rsrc_t& rw, const bf16_t* dH, const bf16_t* hd, const float* hw,
                                          int row0, int B, int Tn) {
  if constexpr (GEN) {
    rs = tile_rsrc(hd, row0, B, 1, 1);
    rw = make_rsrc(hw, hw ? Tn * W * 4 : 0);
  } else {
    rs = tile_rsrc(dH, row0, B, Tn, W);
    rw = make_rsrc(nullptr, 0);
  }
}

template <int W>
__device__ __forceinline__ void tile8_store(const bf16_t* buf, int LD, rsrc_t rd, int Tn, int t, bool on, int ltid) {
  constexpr int CPR = W / 4, NJ = (32 * CPR + 255) / 256;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int e = ltid + 256 * j;
    const int r = e / CPR, c = e - r * CPR;
    const bool ok = r < 32;
    const v2i v = *reinterpret_cast<const v2i*>(buf + (ok ? r : 31) * LD + 4 * c);
    __builtin_amdgcn_raw_buffer_store_b64(v, rd, (on && ok) ? (r * Tn * W + 4 * c) * 2 : kOOB, t * W * 2, 0);
  }
}

}  // namespace

// ==========================================================================================
// tangent forward at the taped primal point: zdot_t = xdot_t W + hdot_{t-1} U
// ==========================================================================================
template <int H, int ACT, int KX, int TILES>
__global__ void __launch_bounds__(256 * TILES)
lstm_tfwd2_kernel(const bf16_t* __restrict__ xd, const float* __restrict__ W, const float* __restrict__ U,
                  const bf16_t* __restrict__ tape, bf16_t* __restrict__ hds, bf16_t* __restrict__ ttape, int B, int Tn,
                  int K_rt) {
  constexpr int act = ACT;
  using P = MF<bf16_t>;
  constexpr int G = 4 * H, NKH = (H + 15) / 16, LH = NKH * 16 + 8, KPADH = NKH * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int K = KX ? KX : K_rt;
  const int KP = (K + 15) & ~15, LX = KP + 8, NKX = KP / 16;
  const int tile = threadIdx.x >> 8, ltid = threadIdx.x & 255;
  bf16_t* Wt = reinterpret_cast<bf16_t*>(smem);
  bf16_t* xb = Wt + G * LX + tile * (2 * 32 * LX + 2 * 32 * LH);
  bf16_t* hb = xb + 2 * 32 * LX;
  const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) & 3;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // wave index as a scalar (uniform offsets)
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int uc = uok ? u : H - 1;
  const int nrb = (B + 31) / 32, ngrp = (nrb + TILES - 1) / TILES;

  stage_wt(Wt, W, K, G, LX);
  for (int i = ltid; i < 2 * 32 * LX; i += 256) xb[i] = 0;
  typename P::frag ub[4][NKH];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int ks = 0; ks < NKH; ++ks)
      ub[q][ks] = P::make([&](int k) {
        const float v = U[min(k, H - 1) * G + q * H + uc];
        return (uok && k < H) ? v : 0.f;
      }, ks, lane);
    __builtin_amdgcn_sched_barrier(0);  // one gate's loads in flight at a time: bounded prologue live range
  }

  for (int grp = blockIdx.x; grp < ngrp; grp += gridDim.x) {
  const int rb = grp * TILES + tile, row0 = rb * 32;
  const rsrc_t rx = tile_rsrc(xd, row0, B, Tn, K), rh = tile_rsrc(hds, row0, B, Tn, H);
  const rsrc_t rt = tape_rsrc(tape, rb, nrb, Tn), rtt = tape_rsrc(ttape, rb, nrb, Tn);  // idle tile: 0 records
  for (int i = ltid; i < 2 * 32 * LH; i += 256) hb[i] = 0;
  float cd[16], cprev[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) { cd[r] = 0.f; cprev[r] = 0.f; }
  XPref pf;
  __syncthreads();
  x_load<KX>(pf, rx, Tn, 0, true, K, ltid);
  x_store_lds<KX>(pf, xb, K, LX, ltid);
  // primal tape of step 0 (gates + cell)
  Slot16 tg[TAPE_SLOTS];
#pragma unroll
  for (int s = 0; s < TAPE_SLOTS; ++s) tg[s] = ld_slot(rt, uok, lane * 8, tape_off(0, wu) + s * SLOT_ELEMS);
  __syncthreads();

  for (int t = 0; t < Tn; ++t) {
    const bf16_t* xcur = xb + (t & 1) * 32 * LX;
    const bf16_t* hcur = hb + (t & 1) * 32 * LH;
    bf16_t* hnext = hb + ((t + 1) & 1) * 32 * LH;
    // next step's x tile and primal tape first, then this tile's pending h stores
    const bool nx = t + 1 < Tn;
    x_load<KX>(pf, rx, Tn, t + 1, nx, K, ltid);
    Slot16 tn[TAPE_SLOTS];
#pragma unroll
    for (int s = 0; s < TAPE_SLOTS; ++s) tn[s] = ld_slot(rt, uok && nx, lane * 8, tape_off(t + 1, wu) + s * SLOT_ELEMS);
    tile8_store<H>(hcur, LH, rh, Tn, t - 1, t > 0, ltid);
    f32x16 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = zero16();
    const bf16_t* xrow = xcur + (lane & 31) * LX;
    for (int kx = 0; kx < NKX; ++kx) {
      const typename P::frag a = P::lda(xrow, kx, lane);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = P::mma(a, P::lda(Wt + (q * H + uc) * LX, kx, lane), acc[q]);
    }
    const bf16_t* hrow = hcur + (lane & 31) * LH;
#pragma unroll
    for (int ks = 0; ks < NKH; ++ks) {
      const typename P::frag a = P::lda(hrow, ks, lane);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = P::mma(a, ub[q][ks], acc[q]);
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      uint32_t pk[TAPE_SLOTS][4];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = half * 8 + i;
        const int rr = acc32_row(r, lane);
        const float ig = tg[0].get(r), fg = tg[1].get(r), gg = tg[2].get(r), og = tg[3].get(r), c = tg[4].get(r);
        const float idot = ig * (1.f - ig) * acc[0][r];
        const float fdot = fg * (1.f - fg) * acc[1][r];
        const float gdot = act_dy(act, gg) * acc[2][r];
        const float odot = og * (1.f - og) * acc[3][r];
        float cdn = fdot * cprev[r] + fg * cd[r] + idot * gg + ig * gdot;
        const float ca = act_f(act, c);
        float hd = odot * ca + og * act_dy(act, ca) * cdn;
        if (!uok) { cdn = 0.f; hd = 0.f; }
        cd[r] = cdn;
        cprev[r] = c;
        if (u < KPADH) hnext[rr * LH + u] = f2bf(hd);
        put4(pk[0], i, acc[0][r]); put4(pk[1], i, acc[1][r]); put4(pk[2], i, acc[2][r]); put4(pk[3], i, acc[3][r]);
        put4(pk[4], i, cdn);
      }
      const int to = tape_off(t, wu) + half * SLOT_HALF;
#pragma unroll
      for (int s = 0; s < TAPE_SLOTS; ++s) st_slot(rtt, uok, lane * 8, to + s * SLOT_ELEMS, pk[s]);
    }
    if (nx) x_store_lds<KX>(pf, xb + ((t + 1) & 1) * 32 * LX, K, LX, ltid);
#pragma unroll
    for (int s = 0; s < TAPE_SLOTS; ++s) tg[s] = tn[s];
    lds_barrier();  // step hand-off: LDS only, stores stay in flight
  }
  tile8_store<H>(hb + (Tn & 1) * 32 * LH, LH, rh, Tn, Tn - 1, true, ltid);
  __syncthreads();
  }
}

// ==========================================================================================
// BPTT v3: role-split workgroup (8 waves, 2 per SIMD).  The v2 BPTT keeps U^T AND W^T fragments in
// one wave (420 registers: one wave per SIMD, nothing hides its latencies).  Here waves 0-3 run
// the recurrence (U^T fragments, tape loads, gate math: dz_t into LDS) and waves 4-7 move data and
// produce the input gradient (W^T fragments: dx_{t+1} = dz_{t+1} W^T, the dz tile copy LDS -> HBM,
// the dH tiles HBM -> LDS two steps ahead).  Each SIMD pairs one wave of each role, so the gate
// math of one overlaps the MFMAs / stores of the other, and the recurrence waves issue only loads
// (their waits never cover a store).  The two roles run separate loops with the same barrier
// sequence (3 per row block + 1 per step).
// ==========================================================================================
// ==========================================================================================
// Tangent reverse v4: 16x16x32 MFMAs, 16 units per wave.
//
// The v2 kernel (32 units per wave, 32x32x16) holds U^T and W^T fragments (200 VGPRs) plus 12
// tape slots, both adjoint accumulators and the carried cell adjoints in one wave: ~500 registers,
// one wave per SIMD, spills in the dX variant, and nothing to hide its latencies.  A role split
// (as BPTT v3) does not fit either: the recurrence alone needs ~290 registers.  Halving the wave's
// column count halves every per-lane array instead: with v_mfma_f32_16x16x32_bf16 a wave owns
// 16 units x 32 rows (U^T / W^T fragments 52 VGPRs each, 8 values per tape slot), so seven
// compute waves (112 units >= H) fit at two waves per SIMD with the input gradient fused, and
// the eighth wave is a data wave: dz / dzdot tile stores and the dH / dHdot tiles HBM -> LDS.
// The compute waves issue tape loads and the dX stores only, loads first.  The tapes keep the
// 32x32 layout written by lstm_fwd2 / lstm_tfwd2: a 16x16 accumulator lane's four rows of one
// 16-row block are four contiguous values of one 32x32 lane's slot half (one 8-byte load).
// ==========================================================================================
// a K extent as full 32-wide k-steps plus at most one 16-wide tail step (v_mfma_f32_16x16x16_bf16):
// K = 100 -> 3 x 32 + 16 = 112 instead of 128 (fewer fragment registers and MFMAs)
template <int KD>
struct KSplit {
  static constexpr bool TAIL = KD > 0 && (KD % 32) != 0 && (KD % 32) <= 16;
  static constexpr int NF = KD > 0 ? (TAIL ? KD / 32 : (KD + 31) / 32) : 4;  // (KD = 0: runtime K <= 128)
  static constexpr int KP = 32 * NF + (TAIL ? 16 : 0);
};
typedef short bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mma16k16(const bf16x4& a, const bf16x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// gfx950 forwards an MFMA accumulator to the next MFMA's SrcC only between SAME opcodes: a
// v_mfma_f32_16x16x16_bf16 reading the result of a v_mfma_f32_16x16x32_bf16 as SrcC reads registers 0-1
// stale below 5 wait states, the reverse pair registers 2-3 (scripts/probes/mfma_srcc_probe.hip,
// profiles/r03_race) -- and LLVM puts as few as 1 (scripts/isa_mfma_srcc.py).  That was the run-to-run
// nondeterminism of rows 4 g + {0, 1} in the bf16 tangent reverse / two-step-prefetch forward
// (profiles/r02_det).  xdl_switch() sits between the two kinds of MFMA of one accumulator chain: no
// instruction crosses it and the chain's last MFMA is >= 5 wait states behind the first of the other
// kind (operand loads are issued before it).
__device__ __forceinline__ void xdl_switch() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
struct Slot8 {  // 8 bf16 of one 16x16-layout lane: block m = 0, 1 (rows 16 m + 4 (lane >> 4) + i)
  uint2 m0, m1;
  __device__ __forceinline__ float get(int m, int i) const {
    const uint32_t w = m == 0 ? ((i >> 1) ? m0.y : m0.x) : ((i >> 1) ? m1.y : m1.x);
    return (i & 1) ? hi_bf(w) : lo_bf(w);
  }
  __device__ __forceinline__ f2_t get2(int m, int p) const {  // rows 2 p, 2 p + 1 of block m
    const uint32_t w = m == 0 ? (p ? m0.y : m0.x) : (p ? m1.y : m1.x);
    return f2_t{lo_bf(w), hi_bf(w)};
  }
};
__device__ __forceinline__ Slot8 ld_slot8(rsrc_t rs, bool on, int lane_off, int uoff) {
  Slot8 s;
  const int v = on ? lane_off * 2 : kOOB;
  s.m0 = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, v, uoff * 2, 0));
  s.m1 = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, v, (uoff + SLOT_HALF) * 2, 0));
  return s;
}
__device__ __forceinline__ f32x4 mma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// dX rows of a 16x16 accumulator pair: 8 two-byte stores per lane, always issued
__device__ __forceinline__ void store_dx16(const f32x4 (&ax)[2], rsrc_t rd, int Tn, int t, bool on, int nr, int K,
                                           int kc, int g4) {
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * m + 4 * g4 + i;
      const int off = (on && kc < K && row < nr) ? (row * Tn * K + kc) * 2 : kOOB;
      __builtin_amdgcn_raw_buffer_store_b16(f2bf(ax[m][i]), rd, off, t * K * 2, 0);
    }
}
// one wave moves a [32 x W] LDS tile to step t of a tile descriptor (16-byte chunks, soffset 0)
template <int W>
__device__ __forceinline__ void tile16_store_w(const bf16_t* buf, int LD, rsrc_t rd, int Tn, int t, bool on, int lane) {
  constexpr int CPR = W / 8, NJ = (32 * CPR + 63) / 64;
#pragma unroll 5
  for (int j = 0; j < NJ; ++j) {
    const int e = lane + 64 * j;
    const int r = e / CPR, c = e - r * CPR;
    const bool ok = r < 32;
    const v4i v = *reinterpret_cast<const v4i*>(buf + (ok ? r : 31) * LD + 8 * c);
    __builtin_amdgcn_raw_buffer_store_b128(v, rd, (on && ok) ? ((r * Tn + t) * W + 8 * c) * 2 : kOOB, 0, 0);
  }
}
// one wave stores a [32 x W] LDS tile to step t of a tile descriptor in 8-byte chunks
template <int W>
__device__ __forceinline__ void tile8_store_w(const bf16_t* buf, int LD, rsrc_t rd, int Tn, int t, bool on, int lane) {
  constexpr int CPR = W / 4, NJ = (32 * CPR + 63) / 64;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int e = lane + 64 * j;
    const int r = e / CPR, c = e - r * CPR;
    const bool ok = r < 32;
    const v2i v = *reinterpret_cast<const v2i*>(buf + (ok ? r : 31) * LD + 4 * c);
    __builtin_amdgcn_raw_buffer_store_b64(v, rd, (on && ok) ? (r * Tn * W + 4 * c) * 2 : kOOB, t * W * 2, 0);
  }
}
// one wave's share of a [32 x W] tile in 8-byte chunks, HBM -> registers -> LDS
template <int W>
struct Tile8w {
  static constexpr int CPR = W / 4, NJ = (32 * CPR + 63) / 64;
  v2i v[NJ];
  __device__ __forceinline__ void load(rsrc_t rs, int Tn, int t, bool on, int lane) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int e = lane + 64 * j;
      const int r = e / CPR, c = e - r * CPR;
      v[j] = __builtin_amdgcn_raw_buffer_load_b64(rs, (on && r < 32) ? (r * Tn * W + 4 * c) * 2 : kOOB, t * W * 2, 0);
    }
  }
  __device__ __forceinline__ void to_lds(bf16_t* buf, int LD, int lane) const {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int e = lane + 64 * j;
      const int r = e / CPR, c = e - r * CPR;
      if (r < 32) *reinterpret_cast<v2i*>(buf + r * LD + 4 * c) = v[j];
    }
  }
};

template <int H>
struct Tb4Geo {
  // the gate axis as full 32-wide k-steps + a 16-wide tail: G = 400 -> 12 x 32 + 16, no padding
  // dz tile row stride: the smallest LG >= KP with (LG / 2) % 64 == 8 dwords, which makes the MFMA
  // A-operand ds_read_b128 (lane l: row l & 15, k-group l >> 4) conflict-free in all four lane
  // groups (scripted bank model, CDNA4 b128 lane groups); KP + 8 (408 at H = 100) was 2-way
  // conflicted in every group (~1.5 conflict cycles per LDS instruction, profiles/r01_fwd5)
  static constexpr int lg_stride(int kp) { return kp + ((16 - kp % 128) + 128) % 128; }
  static constexpr int G = 4 * H, NK = KSplit<G>::NF, KP = KSplit<G>::KP, LG = lg_stride(KP), LH = ((H + 3) / 4) * 4 + 4;
  static_assert((LG / 2) % 64 == 8 && LG >= KP, "dz tile stride");
  static constexpr bool TAIL = KSplit<G>::TAIL;
  static constexpr int NCW = (H + 15) / 16;  // compute waves
  static_assert(NCW <= 7, "tbwd4: H <= 112 (7 compute waves + 1 data wave)");
  static constexpr size_t smem = (size_t)(4 * 32 * LG + 4 * 32 * LH) * 2;
};

// BPTT wave priority.  The compute waves 4-6 share a SIMD with waves 0-2 and, being dispatched second,
// lose VALU arbitration to them on every segment; one s_setprio 1 for them before the loop (no flips
// inside) measured bwd_dx -3.0 % at K = 100 (2.93 -> 2.84 ms, twice), the other BPTT ops unchanged;
// flips around each step's MFMA chain (2): unchanged (profiles/r05_bwdpk/prio).  0: off.
#ifndef HFREP_BWD_PRIO
#define HFREP_BWD_PRIO 1
#endif
#ifndef HFREP_BWD_PK
#define HFREP_BWD_PK 1  // BPTT (TG = false): packed-fp32 cell math (0: the scalar form)
#endif
// a lane's two vertically adjacent bf16 tile values (rows r, r + 1; row stride ld) from one conversion
__device__ __forceinline__ void st_bf_pair(bf16_t* p, int ld, f2_t v) {
  const uint32_t w = pk2bf(v[0], v[1]);
  p[0] = (bf16_t)(w & 0xffffu);
  p[ld] = (bf16_t)(w >> 16);
}
#ifndef HFREP_BWD_PREFETCH
#define HFREP_BWD_PREFETCH 1  // BPTT (TG = false): tape slots one step ahead (0: loaded at the top of their step)
#endif
template <int H, int ACT, bool DX, bool GEN = false, bool TG = true>
__global__ void __launch_bounds__(512)
lstm_tbwd4_kernel(const bf16_t* __restrict__ dH, const bf16_t* __restrict__ dHd, const bf16_t* __restrict__ tape,
                  const bf16_t* __restrict__ ttape, const float* __restrict__ U, bf16_t* __restrict__ dZ,
                  bf16_t* __restrict__ dZd, const float* __restrict__ W, bf16_t* __restrict__ dX,
                  bf16_t* __restrict__ dXd, int B, int Tn, int K, const bf16_t* __restrict__ hd,
                  const bf16_t* __restrict__ hdd, const float* __restrict__ hw) {
  constexpr int act = ACT;
  using Geo = Tb4Geo<H>;
  constexpr int G = Geo::G, NK = Geo::NK, KP = Geo::KP, LG = Geo::LG, LH = Geo::LH;
  constexpr bool TAIL = Geo::TAIL;
  constexpr bool PF = !TG && HFREP_BWD_PREFETCH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* zb = reinterpret_cast<bf16_t*>(smem);  // [2][32][LG]  dz_t
  bf16_t* zdb = zb + 2 * 32 * LG;                 // [2][32][LG]  dzdot_t
  bf16_t* dhb = zdb + 2 * 32 * LG;                // [2][32][LH]  dH_t
  bf16_t* dhdb = dhb + 2 * 32 * LH;               // [2][32][LH]  dHdot_t
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nrb = (B + 31) / 32;
  // K padding columns [G, KP) of the dz tiles (if any) are read by the last MFMA k-step: zero them
  // once (nothing writes them afterwards; garbage there could be a NaN times a zero fragment)
  if constexpr (KP > G) {
    for (int i = threadIdx.x; i < 4 * 32 * (KP - G); i += 512) {
      const int buf = i / (32 * (KP - G)), rem = i - buf * 32 * (KP - G);
      const int r = rem / (KP - G), c = G + rem - r * (KP - G);
      zb[buf * 32 * LG + r * LG + c] = 0;  // buf 0..3 spans zb[0..1] and zdb[0..1]
    }
  }

  if (wave < Geo::NCW) {
    // ---------------- compute waves: 16 units each ----------------
    const int g4 = lane >> 4, c = 16 * wave + (lane & 15);
    const bool uok = c < H;
    const int wt32 = __builtin_amdgcn_readfirstlane(wave >> 1);  // the 32x32 tape wave holding unit c
    const int lo8 = (32 * (g4 & 1) + (c & 31)) * 8 + 4 * (g4 >> 1);
    bf16x8 ut[NK];
    bf16x4 ut4;  // 16-wide tail step (4 values per lane: k = 32 NK + 4 (lane >> 4) + j)
#pragma unroll
    for (int ks = 0; ks < NK; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * ks + 8 * g4 + j;
        const float v = U[(size_t)(uok ? c : H - 1) * G + min(k, G - 1)];
        ut[ks][j] = (short)f2bf((uok && k < G) ? v : 0.f);
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 32 * NK + 4 * g4 + j;
      ut4[j] = (short)f2bf((TAIL && uok && k < G) ? U[(size_t)(uok ? c : H - 1) * G + min(k, G - 1)] : 0.f);
    }
    const bool xw = DX && 16 * wave < K;  // this wave owns input columns (wave-uniform)
    bf16x8 wt[DX ? NK : 1];
    bf16x4 wt4;
    if constexpr (DX) {
#pragma unroll
      for (int ks = 0; ks < NK; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * ks + 8 * g4 + j;
          const float v = W[(size_t)min(c, K - 1) * G + min(k, G - 1)];
          wt[ks][j] = (short)f2bf((c < K && k < G) ? v : 0.f);
        }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 32 * NK + 4 * g4 + j;
        wt4[j] = (short)f2bf((TAIL && c < K && k < G) ? W[(size_t)min(c, K - 1) * G + min(k, G - 1)] : 0.f);
      }
    }
    // (HFREP_BWD_PRIO, BPTT only: 1 = the younger compute waves 4-6 at priority 1 for the whole kernel,
    // 2 = priority 1 around each step's MFMA chain; readfirstlane keeps the guard a scalar branch)
    if constexpr (!TG && HFREP_BWD_PRIO == 1)
      if (__builtin_amdgcn_readfirstlane(wave) >= 4) __builtin_amdgcn_s_setprio(1);
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      const int row0 = rb * 32, nr = min(32, B - row0);
      const rsrc_t rt = tape_rsrc(tape, rb, nrb, Tn), rtt = tape_rsrc(ttape, rb, nrb, Tn);
      const rsrc_t rdx = tile_rsrc(DX ? dX : nullptr, row0, B, Tn, DX ? K : 1);
      const rsrc_t rdxd = tile_rsrc(DX ? dXd : nullptr, row0, B, Tn, DX ? K : 1);
      float ac[8], acd[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { ac[e] = 0.f; acd[e] = 0.f; }
      Slot8 cc = ld_slot8(rt, uok, lo8, tape_off(Tn - 1, wt32) + 4 * SLOT_ELEMS);
      Slot8 cdc = {};
      if constexpr (TG) cdc = ld_slot8(rtt, uok, lo8, tape_off(Tn - 1, wt32) + 4 * SLOT_ELEMS);
      // BPTT (PF): the tape slots of step t - 1 are loaded during step t (registers free at TG = false),
      // so their HBM latency hides under a whole step instead of under the step's MFMA chain only
      Slot8 pg[PF ? 4 : 1], pcp = {};
      if constexpr (PF) {
#pragma unroll
        for (int s = 0; s < 4; ++s) pg[s] = ld_slot8(rt, uok, lo8, tape_off(Tn - 1, wt32) + s * SLOT_ELEMS);
        pcp = ld_slot8(rt, uok && Tn > 1, lo8, tape_off(max(Tn - 2, 0), wt32) + 4 * SLOT_ELEMS);
      }
      __syncthreads();  // (A) LDS free (previous row block stored)
      __syncthreads();  // (B) dH_{T-1} / dHd_{T-1} staged
      for (int t = Tn - 1; t >= 0; --t) {
        const int cb = t & 1, nb = (t + 1) & 1;
        const bool pv = t > 0, live = t < Tn - 1;
        Slot8 tg[4], zd[TG ? 4 : 1], cp, cdp = {};
        if constexpr (PF) {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            tg[s] = pg[s];
            pg[s] = ld_slot8(rt, uok && pv, lo8, tape_off(max(t - 1, 0), wt32) + s * SLOT_ELEMS);
          }
          cp = pcp;
          pcp = ld_slot8(rt, uok && t > 1, lo8, tape_off(max(t - 2, 0), wt32) + 4 * SLOT_ELEMS);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            tg[s] = ld_slot8(rt, uok, lo8, tape_off(t, wt32) + s * SLOT_ELEMS);
            if constexpr (TG) zd[s] = ld_slot8(rtt, uok, lo8, tape_off(t, wt32) + s * SLOT_ELEMS);
          }
          cp = ld_slot8(rt, uok && pv, lo8, tape_off(max(t - 1, 0), wt32) + 4 * SLOT_ELEMS);
          if constexpr (TG) cdp = ld_slot8(rtt, uok && pv, lo8, tape_off(max(t - 1, 0), wt32) + 4 * SLOT_ELEMS);
        }
        f32x4 ah[2], ahd[2], ax[2], axd[2];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          ah[m] = f32x4{0.f, 0.f, 0.f, 0.f}; ahd[m] = ah[m]; ax[m] = ah[m]; axd[m] = ah[m];
        }
        if constexpr (!TG && HFREP_BWD_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        if (live) {
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            const bf16_t* rowz = zb + nb * 32 * LG + (16 * m + (lane & 15)) * LG;
            const bf16_t* rowd = zdb + nb * 32 * LG + (16 * m + (lane & 15)) * LG;
            const bf16_t* arow = rowz + 8 * g4;
            const bf16_t* drow = rowd + 8 * g4;
            if (xw) {
#pragma unroll
              for (int ks = 0; ks < NK; ++ks) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(arow + 32 * ks);
                ah[m] = mma16(a, ut[ks], ah[m]);
                if constexpr (DX) ax[m] = mma16(a, wt[ks], ax[m]);
                if constexpr (TG) {
                  const bf16x8 ad = *reinterpret_cast<const bf16x8*>(drow + 32 * ks);
                  ahd[m] = mma16(ad, ut[ks], ahd[m]);
                  if constexpr (DX) axd[m] = mma16(ad, wt[ks], axd[m]);
                }
              }
              if constexpr (TAIL) {
                const bf16x4 a = *reinterpret_cast<const bf16x4*>(rowz + 32 * NK + 4 * g4);
                const bf16x4 ad = TG ? *reinterpret_cast<const bf16x4*>(rowd + 32 * NK + 4 * g4) : a;
                xdl_switch();
                ah[m] = mma16k16(a, ut4, ah[m]);
                if constexpr (TG) ahd[m] = mma16k16(ad, ut4, ahd[m]);
                if constexpr (DX) {
                  ax[m] = mma16k16(a, wt4, ax[m]);
                  if constexpr (TG) axd[m] = mma16k16(ad, wt4, axd[m]);
                }
              }
            } else {
#pragma unroll
              for (int ks = 0; ks < NK; ++ks) {
                ah[m] = mma16(*reinterpret_cast<const bf16x8*>(arow + 32 * ks), ut[ks], ah[m]);
                if constexpr (TG) ahd[m] = mma16(*reinterpret_cast<const bf16x8*>(drow + 32 * ks), ut[ks], ahd[m]);
              }
              if constexpr (TAIL) {
                const bf16x4 a = *reinterpret_cast<const bf16x4*>(rowz + 32 * NK + 4 * g4);
                const bf16x4 ad = TG ? *reinterpret_cast<const bf16x4*>(rowd + 32 * NK + 4 * g4) : a;
                xdl_switch();
                ah[m] = mma16k16(a, ut4, ah[m]);
                if constexpr (TG) ahd[m] = mma16k16(ad, ut4, ahd[m]);
              }
            }
          }
        }
        if constexpr (!TG && HFREP_BWD_PRIO == 2) __builtin_amdgcn_s_setprio(0);
        if constexpr (DX) {
          store_dx16(ax, rdx, Tn, t + 1, xw && live, nr, K, c, g4);
          if constexpr (TG) store_dx16(axd, rdxd, Tn, t + 1, xw && live, nr, K, c, g4);
        }
        const bf16_t* dh_t = dhb + cb * 32 * LH;
        const bf16_t* dhd_t = dhdb + cb * 32 * LH;
        if constexpr (!TG && HFREP_BWD_PK) {
          // BPTT only (the former lstm_bwd3's contract): dz from the output adjoint and the carried cell adjoint.
          // Packed: rows 2 p, 2 p + 1 of a lane's four go through v_pk_mul / v_pk_add / v_pk_fma_f32 together,
          // act(c) as exp2 + rcp without abs / copysign, and the two rows' dz share one v_cvt_pk_bf16_f32
          // (low half -> row rr, high half -> row rr + 1).  The scalar form issued ~17 VALU per MFMA.
          constexpr float CS = act_prescale<ACT>();
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
              const int e = 4 * m + 2 * p, rr = 16 * m + 4 * g4 + 2 * p;
              const f2_t ig = tg[0].get2(m, p), fg = tg[1].get2(m, p), gg = tg[2].get2(m, p), og = tg[3].get2(m, p);
              const f2_t cv = cc.get2(m, p), cpv = cp.get2(m, p);
              const f2_t dh = uok ? f2_t{bf2f(dh_t[rr * LH + c]), bf2f(dh_t[(rr + 1) * LH + c])} : f2_t{0.f, 0.f};
              const f2_t a_h = dh + f2_t{ah[m][2 * p], ah[m][2 * p + 1]};
              const f2_t ca = act_s2<ACT>(CS * cv);
              const f2_t dov = a_h * ca;
              const f2_t dct = f2_t{ac[e], ac[e + 1]} + a_h * og * act_dy2<ACT>(ca);
              const f2_t an = dct * fg;
              ac[e] = uok ? an[0] : 0.f;
              ac[e + 1] = uok ? an[1] : 0.f;
              if (uok) {
                bf16_t* zr = zb + cb * 32 * LG + rr * LG + c;
                st_bf_pair(zr, LG, dct * gg * (ig - ig * ig));
                st_bf_pair(zr + H, LG, dct * cpv * (fg - fg * fg));
                st_bf_pair(zr + 2 * H, LG, dct * ig * act_dy2<ACT>(gg));
                st_bf_pair(zr + 3 * H, LG, dov * (og - og * og));
              }
            }
        } else if constexpr (!TG) {
          // (scalar form, HFREP_BWD_PK=0)
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int e = 4 * m + i, rr = 16 * m + 4 * g4 + i;
              const float ig = tg[0].get(m, i), fg = tg[1].get(m, i), gg = tg[2].get(m, i), og = tg[3].get(m, i);
              const float cv = cc.get(m, i), cpv = cp.get(m, i);
              const float a_h = (uok ? bf2f(dh_t[rr * LH + c]) : 0.f) + ah[m][i];
              const float ca = act_f(act, cv);
              const float dov = a_h * ca;
              const float dct = ac[e] + a_h * og * act_dy(act, ca);
              ac[e] = uok ? dct * fg : 0.f;
              if (uok) {
                bf16_t* zr = zb + cb * 32 * LG + rr * LG + c;
                zr[0] = f2bf(dct * gg * ig * (1.f - ig));
                zr[H] = f2bf(dct * cpv * fg * (1.f - fg));
                zr[2 * H] = f2bf(dct * ig * act_dy(act, gg));
                zr[3 * H] = f2bf(dov * og * (1.f - og));
              }
            }
        } else {
  #pragma unroll
          for (int m = 0; m < 2; ++m)
  #pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int e = 4 * m + i, rr = 16 * m + 4 * g4 + i;
              const float ig = tg[0].get(m, i), fg = tg[1].get(m, i), gg = tg[2].get(m, i), og = tg[3].get(m, i);
              const float cv = cc.get(m, i), cpv = cp.get(m, i), cd = cdc.get(m, i), cdpv = cdp.get(m, i);
              const float zdi = zd[0].get(m, i), zdf = zd[1].get(m, i), zdg = zd[2].get(m, i), zdo = zd[3].get(m, i);
              const float si = ig * (1.f - ig), sf = fg * (1.f - fg), so = og * (1.f - og);
              const float sg = act_dy(act, gg);
              const float idot = si * zdi, fdot = sf * zdf, gdot = sg * zdg, odot = so * zdo;
              const float ca = act_f(act, cv);
              const float e1 = act_dy(act, ca), e2 = act_d2y(act, ca);
              const float a_h = (uok ? bf2f(dh_t[rr * LH + c]) : 0.f) + ah[m][i];
              const float a_hd = (uok ? bf2f(dhd_t[rr * LH + c]) : 0.f) + ahd[m][i];
              const float a_od = a_hd * ca;
              const float a_o = a_h * ca + a_hd * e1 * cd;
              const float a_cd = acd[e] + a_hd * og * e1;
              const float a_c = ac[e] + a_h * og * e1 + a_hd * (odot * e1 + og * e2 * cd);
              const float a_fd = a_cd * cpv, a_id = a_cd * gg, a_gd = a_cd * ig;
              const float a_f = a_c * cpv + a_cd * cdpv;
              const float a_i = a_c * gg + a_cd * gdot;
              const float a_g = a_c * ig + a_cd * idot;
              ac[e] = uok ? a_c * fg + a_cd * fdot : 0.f;
              acd[e] = uok ? a_cd * fg : 0.f;
              const float s2i = si * (1.f - 2.f * ig), s2f = sf * (1.f - 2.f * fg), s2o = so * (1.f - 2.f * og);
              const float s2g = act_d2y(act, gg);
              if (uok) {
                bf16_t* zr = zb + cb * 32 * LG + rr * LG + c;
                bf16_t* dr = zdb + cb * 32 * LG + rr * LG + c;
                zr[0] = f2bf(a_i * si + a_id * s2i * zdi);
                zr[H] = f2bf(a_f * sf + a_fd * s2f * zdf);
                zr[2 * H] = f2bf(a_g * sg + a_gd * s2g * zdg);
                zr[3 * H] = f2bf(a_o * so + a_od * s2o * zdo);
                dr[0] = f2bf(a_id * si);
                dr[H] = f2bf(a_fd * sf);
                dr[2 * H] = f2bf(a_gd * sg);
                dr[3 * H] = f2bf(a_od * so);
              }
            }
        }
        cc = cp;
        if constexpr (TG) cdc = cdp;
        lds_barrier();  // step hand-off
      }
      if constexpr (DX) {  // dx_0 / dxdot_0 from the last dz tiles (final after the last barrier)
        f32x4 ax[2], axd[2];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          ax[m] = f32x4{0.f, 0.f, 0.f, 0.f}; axd[m] = ax[m];
          if (xw) {
            const bf16_t* rowz = zb + (16 * m + (lane & 15)) * LG;
            const bf16_t* rowd = zdb + (16 * m + (lane & 15)) * LG;
#pragma unroll
            for (int ks = 0; ks < NK; ++ks) {
              ax[m] = mma16(*reinterpret_cast<const bf16x8*>(rowz + 8 * g4 + 32 * ks), wt[ks], ax[m]);
              if constexpr (TG) axd[m] = mma16(*reinterpret_cast<const bf16x8*>(rowd + 8 * g4 + 32 * ks), wt[ks], axd[m]);
            }
            if constexpr (TAIL) {
              const bf16x4 a = *reinterpret_cast<const bf16x4*>(rowz + 32 * NK + 4 * g4);
              const bf16x4 ad = TG ? *reinterpret_cast<const bf16x4*>(rowd + 32 * NK + 4 * g4) : a;
              xdl_switch();
              ax[m] = mma16k16(a, wt4, ax[m]);
              if constexpr (TG) axd[m] = mma16k16(ad, wt4, axd[m]);
            }
          }
        }
        store_dx16(ax, rdx, Tn, 0, xw, nr, K, c, g4);
        if constexpr (TG) store_dx16(axd, rdxd, Tn, 0, xw, nr, K, c, g4);
      }
      __syncthreads();  // (C)
    }
  } else if (wave == 7) {
    // ---------------- data wave ----------------
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      const int row0 = rb * 32;
      const rsrc_t rz = tile_rsrc(dZ, row0, B, Tn, G), rzd = tile_rsrc(dZd, row0, B, Tn, G);
      rsrc_t rdh, rdhd, rhw;
      head_rsrc<H, GEN>(rdh, rhw, dH, hd, hw, row0, B, Tn);
      head_rsrc<H, GEN>(rdhd, rhw, dHd, hdd, hw, row0, B, Tn);
      TileSrc<H, 64, GEN> a, ad;
      a.load(rdh, rhw, Tn, Tn - 1, true, lane);
      if constexpr (TG) ad.load(rdhd, rhw, Tn, Tn - 1, true, lane);
      __syncthreads();  // (A)
      a.to_lds(dhb + ((Tn - 1) & 1) * 32 * LH, LH, lane);
      if constexpr (TG) ad.to_lds(dhdb + ((Tn - 1) & 1) * 32 * LH, LH, lane);
      __syncthreads();  // (B)
      for (int t = Tn - 1; t >= 0; --t) {
        const int nb = (t + 1) & 1;
        const bool pv = t > 0, live = t < Tn - 1;
        a.load(rdh, rhw, Tn, t - 1, pv, lane);  // loads first: their wait covers no store of this step
        if constexpr (TG) ad.load(rdhd, rhw, Tn, t - 1, pv, lane);
        tile16_store_w<G>(zb + nb * 32 * LG, LG, rz, Tn, t + 1, live, lane);
        if constexpr (TG) tile16_store_w<G>(zdb + nb * 32 * LG, LG, rzd, Tn, t + 1, live, lane);
        if (pv) {
          a.to_lds(dhb + nb * 32 * LH, LH, lane);  // dH_{t-1}: (t - 1) & 1 == nb
          if constexpr (TG) ad.to_lds(dhdb + nb * 32 * LH, LH, lane);
        }
        lds_barrier();
      }
      tile16_store_w<G>(zb, LG, rz, Tn, 0, true, lane);
      if constexpr (TG) tile16_store_w<G>(zdb, LG, rzd, Tn, 0, true, lane);
      __syncthreads();  // (C)
    }
  } else {
    // idle waves (H <= 96): keep the barrier sequence
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      __syncthreads();
      __syncthreads();
      for (int t = Tn - 1; t >= 0; --t) lds_barrier();
      __syncthreads();
    }
  }
}

// ==========================================================================================
// Forward / tangent forward v4: 16x16x32 MFMAs, 16 units per wave, 7 compute waves + 1 data wave.
//
// Same decomposition as the tangent reverse v4: a compute wave owns 16 units of one 32-row tile
// and keeps BOTH weight operands as register fragments (W^T for the input projection, U^T for
// the recurrence: 4 gates x ceil(K/32) and 4 gates x 4 k-steps of 8 bf16), so the step loop reads
// only the x / h tiles from LDS (v2 re-read the staged W^T from LDS every step: 28 KB per wave per
// step).  The data wave streams x_{t+1} (or xdot_{t+1}) HBM -> LDS and h_{t-1} (hdot) LDS -> HBM;
// the compute waves issue only the tape stores (and, for the tangent, the primal tape loads one
// step ahead).  Tapes are written in the 32x32 layout the BPTT / tangent reverse kernels read: a
// lane's four rows of a 16-row block are four contiguous values of a slot half (8-byte stores).
// TAN = false: z = x W + h U + b, tape = gate activations + cell.  TAN = true: zdot = xdot W +
// hdot U at the taped primal point, tape = tangent pre-activations + cell tangent.
// ==========================================================================================
// One step's tape image of a row block (NW2 x TAPE_SLOTS slots of 2 KiB, already in the global
// blocked layout) LDS -> HBM by ONE wave: 16-byte lane stores, each wave instruction one contiguous
// KiB.  The compute waves used to store their own 8-byte pieces (two 256-byte runs per instruction):
// those stores ran at 4.8 TB/s against 6.1 for 16-byte ones (scripts/probes/store_probe.hip) and,
// worse, stalled the compute waves at issue, so tape traffic and the recurrence did not overlap.
// Lanes of padded units (unit >= H) get the out-of-range offset: no bytes written for them.
constexpr int FW4_STAGE = NW2 * TAPE_SLOTS * SLOT_ELEMS;
constexpr int TAPE_STORE_AUX = 2;  // cache-policy bits of the tape stream: 2 = nt (non-temporal)
template <int H>
__device__ __forceinline__ void tape_image_store(const bf16_t* img, rsrc_t rt, int t, bool on, int lane) {
  constexpr int NCH = FW4_STAGE / 512, G = 5;  // 1 KiB chunks, stored in groups of G
  static_assert(NCH % G == 0, "chunk groups");
  const int base = t * FW4_STAGE * 2 + lane * 16;
#pragma unroll
  for (int g = 0; g < NCH; g += G) {
    v4i d[G];
#pragma unroll
    for (int j = 0; j < G; ++j) d[j] = *reinterpret_cast<const v4i*>(img + (g + j) * 512 + lane * 8);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int ch = g + j, w = ch / (TAPE_SLOTS * 2);
      const bool ok = on && 32 * w + (lane & 31) < H;
      // 16-byte store: the whole offset in voffset, soffset 0 (see the store-data hazard note);
      // non-temporal (aux 2 = nt): the tape is read back only by the reverse kernels, long after;
      // under the nt policy the concurrent x reads of the recurrence wait less behind it (tape
      // forward 2.72 -> 2.55 ms, tangent 3.33 -> 3.03 ms at B = 262144; sc1 / sc0 sc1: no gain;
      // nt on the reverse kernels' dZ stores: BPTT +8 %; nt tape loads: tangent reverse +3-4 %.  profiles/archive_scripts/gpu_store_policy.sh,
      // profiles/archive_scripts/gpu_ab_lstm.sh, profiles/r01_fwd5/store_policy.jsonl)
      __builtin_amdgcn_raw_buffer_store_b128(d[j], rt, ok ? base + ch * 1024 : kOOB, 0, TAPE_STORE_AUX);
    }
  }
}

// x / h tile row stride (bf16 elements) of the forward: the smallest L >= KP with L % 32 == 16, i.e. a
// row stride of 8 mod 16 dwords, makes the MFMA A-operand ds_read_b128 (lane l: row l & 15, k-group l >> 4)
// conflict-free in all four CDNA4 lane groups (4 LDS cycles instead of 8); the 16-wide tail's ds_read_b64
// becomes 2-way (4 instead of 2), a net 104 -> 64 modelled LDS cycles per wave and step at K = H = 100
// (KP + 8 = 120 was 2-way on every b128 read).  Measured: op times unchanged, and the PMC conflict metric
// (1.5-1.9 cycles per LDS-active cycle) did not move either -- the counted conflicts are in the other LDS
// traffic (profiles/r05_pmc/README.md).  HFREP_FW4_STRIDE=0 restores KP + 8 for A/B.
#ifndef HFREP_FW4_STRIDE
#define HFREP_FW4_STRIDE 1
#endif
__host__ __device__ constexpr int fw4_stride(int kp) { return HFREP_FW4_STRIDE ? kp + ((16 - kp % 32) + 32) % 32 : kp + 8; }
template <int H, int KX>
struct Fw4Geo {
  static constexpr int G = 4 * H, KPH = KSplit<H>::KP, LH = fw4_stride(KPH);
};
// x tile loader, split over the NP compute waves: part p moves chunks j = p, p + NP, ... of the
// tile (8-byte chunks if K % 4 == 0, else 2-byte), i.e. one to three loads per lane per step.
// The per-lane global / LDS offsets do not depend on the step: they are computed once per row
// block (set), so the step loop holds no integer division and no lane-dependent branch (an
// exec-masked form let the compiler sink the loads into divergent blocks and corrupt values of
// the tangent forward).  Chunks past the tile load from kOOB (zeros) into an LDS trash word.
template <int KX, int NP>
struct XPart {
  static constexpr bool VEC = KX > 0 && KX % 4 == 0;
  static constexpr int NJT = VEC ? (32 * (KX / 4) + 63) / 64 : (32 * (KX ? KX : 128) + 63) / 64;  // whole tile
  static constexpr int NJ = (NJT + NP - 1) / NP;                                                  // this part
  uint32_t v[VEC ? 2 * NJ : NJ];
  int goff[NJ], loff[NJ];  // byte offset in the row tile at t = 0 (kOOB: none); LDS element offset (-1: trash)
  __device__ __forceinline__ void set(int Tn, int K, int p, int lane) {
    if constexpr (KX > 0) K = KX;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int j = p + NP * jj, e = lane + 64 * j;
      const int per = VEC ? K / 4 : K, w = VEC ? 4 : 1;
      const int r = e / per, c = e - r * per;
      const bool ok = j < NJT && r < 32;
      goff[jj] = ok ? (r * Tn * K + w * c) * 2 : kOOB;
      loff[jj] = ok ? (r << 16) | (w * c) : -1;
    }
  }
  __device__ __forceinline__ void load(rsrc_t rx, int t, bool on, int K) {
    if constexpr (KX > 0) K = KX;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int vo = on ? goff[jj] : kOOB;
      if constexpr (VEC) {
        const v2i d = __builtin_amdgcn_raw_buffer_load_b64(rx, vo, t * K * 2, 0);
        v[2 * jj] = (uint32_t)d[0];
        v[2 * jj + 1] = (uint32_t)d[1];
      } else {
        v[jj] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rx, vo, t * K * 2, 0);
      }
    }
  }
  __device__ __forceinline__ void to_lds(bf16_t* xb, bf16_t* trash, int LX) const {
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int lo = loff[jj];
      bf16_t* dst = lo >= 0 ? xb + (lo >> 16) * LX + (lo & 0xffff) : trash;
      if constexpr (VEC) *reinterpret_cast<uint2*>(dst) = make_uint2(v[2 * jj], v[2 * jj + 1]);
      else *dst = (bf16_t)v[jj];
    }
  }
};

// HFREP_TFWD4_SIGMOID=1 (diagnosis builds only) routes act = sigmoid's tangent forward to this kernel
// instead of lstm_tfwd2: on it act = sigmoid drifts run to run in rows 30 / 31 of a few row blocks, a
// timing-shaped fault that tanh / linear never show, not even under the perturbations that multiply the
// sigmoid drift (profiles/r05_race/README.md, round-6 section).  The round-5 diagnosis instrumentation of
// this kernel (in-kernel re-check, fingerprint trace, perturbation probes, tail nops) is retired: its
// results are recorded there and the builds live in git history (commit d3e5e5a).
#ifndef HFREP_TFWD4_SIGMOID
#define HFREP_TFWD4_SIGMOID 0
#endif
template <int H, int ACT, int KX, bool TAPE, bool TAN>
__global__ void __launch_bounds__(512)
lstm_fwd4_kernel(const bf16_t* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                 const float* __restrict__ U, const bf16_t* __restrict__ ptape, bf16_t* __restrict__ hs,
                 bf16_t* __restrict__ tape, int B, int Tn, int K_rt, int dbg) {
  constexpr int act = ACT;
  using Geo = Fw4Geo<H, KX>;
  using KS = KSplit<KX>;
  using HS = KSplit<H>;
  constexpr int G = Geo::G, LH = Geo::LH;
  constexpr int NCW = (H + 15) / 16;
  static_assert(NCW <= 7, "fwd4: H <= 112");
  const int K = KX ? KX : K_rt;
  const int KP = KX ? KS::KP : (K + 31) & ~31, LX = fw4_stride(KP), NKX = KX ? KS::NF : KP / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* xb = reinterpret_cast<bf16_t*>(smem);  // [2][32][LX]
  bf16_t* hb = xb + 2 * 32 * LX;                  // [2][32][LH]
  bf16_t* tsg = hb + 2 * 32 * LH;                 // TAPE: [2][NW2 x TAPE_SLOTS x SLOT_ELEMS] step images
  bf16_t* trash = tsg + (TAPE ? 2 * FW4_STAGE : 0);  // 16 bytes nobody reads
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nrb = (B + 31) / 32;
  // K / H padding columns of both tile buffers stay zero (the data wave writes K columns, the
  // compute waves write units < H)
  for (int i = threadIdx.x; i < 2 * 32 * LX; i += 512) xb[i] = 0;
  for (int i = threadIdx.x; i < 2 * 32 * LH; i += 512) hb[i] = 0;
  __syncthreads();

  if (wave < NCW) {
    const int g4 = lane >> 4, c = 16 * wave + (lane & 15);
    const bool uok = c < H;
    const int cc_ = uok ? c : H - 1;
    const int wt32 = __builtin_amdgcn_readfirstlane(wave >> 1);
    const int lo8 = (32 * (g4 & 1) + (c & 31)) * 8 + 4 * (g4 >> 1);
    // register fragments: B[k][n = unit] = W[k][q H + c] (input projection), U[k][q H + c];
    // full 32-wide k-steps (8 values per lane) + an optional 16-wide tail (4 values per lane)
    constexpr int NKXM = KS::NF, NKH = HS::NF;
    bf16x8 wf[4][NKXM], uf[4][NKH];
    bf16x4 wf4[4], uf4[4];
    // forward: gate q's weights and bias are pre-scaled for the packed gate math (act_s2)
    constexpr float SIG = act_prescale<ACT_SIGMOID>(), GSC = act_prescale<ACT>();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float sc = TAN ? 1.f : (q == 2 ? GSC : SIG);
#pragma unroll
      for (int ks = 0; ks < NKXM; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * ks + 8 * g4 + j;
          const float v = W[(size_t)min(k, K - 1) * G + q * H + cc_];
          wf[q][ks][j] = (short)f2bf((uok && k < K) ? v * sc : 0.f);
        }
#pragma unroll
      for (int ks = 0; ks < NKH; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * ks + 8 * g4 + j;
          const float v = U[(size_t)min(k, H - 1) * G + q * H + cc_];
          uf[q][ks][j] = (short)f2bf((uok && k < H) ? v * sc : 0.f);
        }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kx = 32 * NKXM + 4 * g4 + j, kh = 32 * NKH + 4 * g4 + j;
        const float vx = W[(size_t)min(kx, K - 1) * G + q * H + cc_];
        const float vh = U[(size_t)min(kh, H - 1) * G + q * H + cc_];
        wf4[q][j] = (short)f2bf((KS::TAIL && uok && kx < K) ? vx * sc : 0.f);
        uf4[q][j] = (short)f2bf((HS::TAIL && uok && kh < H) ? vh * sc : 0.f);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    float bq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[q] = (!TAN && uok && bias) ? bias[q * H + c] * (q == 2 ? GSC : SIG) : 0.f;
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      const rsrc_t rp = tape_rsrc(TAN ? ptape : nullptr, rb, nrb, Tn);
      float cs[8], cprev[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { cs[e] = 0.f; cprev[e] = 0.f; }
      Slot8 tg[TAN ? TAPE_SLOTS : 1], tn[TAN ? TAPE_SLOTS : 1];
      if constexpr (TAN) {
#pragma unroll
        for (int s = 0; s < TAPE_SLOTS; ++s) tg[s] = ld_slot8(rp, uok, lo8, tape_off(0, wt32) + s * SLOT_ELEMS);
      }
      const rsrc_t rx = tile_rsrc(x, rb * 32, B, Tn, K);
      XPart<KX, NCW> xp;
      xp.set(Tn, K, wave, lane);
      xp.load(rx, 0, true, K);
      __syncthreads();  // (A)
      // h_{-1} = 0: this wave's units of buffer 0
      if (uok)
        for (int r = 0; r < 32; r += 4) hb[(r + g4) * LH + c] = 0;
      xp.to_lds(xb, trash, LX);
      __syncthreads();  // (B) x_0 staged, h_{-1} zeroed
      for (int t = 0; t < Tn; ++t) {
        const bf16_t* xcur = xb + (t & 1) * 32 * LX;
        const bf16_t* hcur = hb + (t & 1) * 32 * LH;
        bf16_t* hnext = hb + ((t + 1) & 1) * 32 * LH;
        xp.load(rx, t + 1, t + 1 < Tn && !(dbg & 4), K);  // x_{t+1}: lands during this step
        if constexpr (TAN) {  // primal tape of the next step (loads only; no store precedes them)
#pragma unroll
          for (int s = 0; s < TAPE_SLOTS; ++s)
            tn[s] = ld_slot8(rp, uok && t + 1 < Tn, lo8, tape_off(min(t + 1, Tn - 1), wt32) + s * SLOT_ELEMS);
        }
        f32x4 acc[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) { acc[q][0] = f32x4{0.f, 0.f, 0.f, 0.f}; acc[q][1] = acc[q][0]; }
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const bf16_t* xrow = xcur + (16 * m + (lane & 15)) * LX + 8 * g4;
#pragma unroll
          for (int ks = 0; ks < NKXM; ++ks) {
            if (KX == 0 && ks >= NKX) break;  // (runtime K only; uniform)
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(xrow + 32 * ks);
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q][m] = mma16(a, wf[q][ks], acc[q][m]);
          }
          const bf16_t* hrow = hcur + (16 * m + (lane & 15)) * LH + 8 * g4;
#pragma unroll
          for (int ks = 0; ks < NKH; ++ks) {
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(hrow + 32 * ks);
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q][m] = mma16(a, uf[q][ks], acc[q][m]);
          }
          // the 16-wide tails (lane holds A[row][32 NF + 4 (lane >> 4) + j]) after both 32-wide chains:
          // one opcode switch per accumulator (xdl_switch); the two tails then chain on the same opcode
          // (16x16x16 -> 16x16x16 forwards: scripts/probes/mfma_srcc_probe.hip).  (Merging both tails into
          // one zero-padded 16x16x32 step needs no switch but spilled more at K = 100: bf16 384.3 vs 376.9 ms)
          if constexpr (KS::TAIL || HS::TAIL) {
            const bf16x4 ax4 = *reinterpret_cast<const bf16x4*>(xcur + (16 * m + (lane & 15)) * LX + 32 * NKXM + 4 * g4);
            const bf16x4 ah4 = *reinterpret_cast<const bf16x4*>(hcur + (16 * m + (lane & 15)) * LH + 32 * NKH + 4 * g4);
            xdl_switch();
            if constexpr (KS::TAIL) {
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[q][m] = mma16k16(ax4, wf4[q], acc[q][m]);
            }
            if constexpr (HS::TAIL) {
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[q][m] = mma16k16(ah4, uf4[q], acc[q][m]);
            }
          }
        }
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          uint32_t pk[TAPE_SLOTS][2];
#pragma unroll
          for (int p = 0; p < 2; ++p) {  // rows 16 m + 4 g4 + 2 p + {0, 1}: one packed pair
            const int e = 4 * m + 2 * p, rr = 16 * m + 4 * g4 + 2 * p;
            const f2_t a0 = {acc[0][m][2 * p], acc[0][m][2 * p + 1]}, a1 = {acc[1][m][2 * p], acc[1][m][2 * p + 1]};
            const f2_t a2 = {acc[2][m][2 * p], acc[2][m][2 * p + 1]}, a3 = {acc[3][m][2 * p], acc[3][m][2 * p + 1]};
            const f2_t cp = {cs[e], cs[e + 1]};
            f2_t v0, v1, v2, v3, v4, hv;
            if constexpr (!TAN) {
              // padded units (!uok): zero weights and bias give s = 0 in every gate; with a tanh cell
              // that makes c and h exactly 0, otherwise h is masked (c is never stored for them)
              const f2_t ig = sig_s2(a0 + bq[0]), fg = sig_s2(a1 + bq[1]);
              const f2_t gg = act_s2<ACT>(a2 + bq[2]), og = sig_s2(a3 + bq[3]);
              const f2_t cn = fg * cp + ig * gg;
              f2_t h = og * act_s2<ACT>(GSC * cn);
              if constexpr (ACT != ACT_TANH) h = uok ? h : f2_t{0.f, 0.f};
              cs[e] = cn[0]; cs[e + 1] = cn[1];
              v0 = ig; v1 = fg; v2 = gg; v3 = og; v4 = cn; hv = h;
            } else {
              f2_t hd2, cd2;
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                const int i = 2 * p + u;
                const float ig = tg[0].get(m, i), fg = tg[1].get(m, i), gg = tg[2].get(m, i), og = tg[3].get(m, i);
                const float cv = tg[4].get(m, i);
                const float idot = ig * (1.f - ig) * acc[0][m][i];
                const float fdot = fg * (1.f - fg) * acc[1][m][i];
                const float gdot = act_dy(act, gg) * acc[2][m][i];
                const float odot = og * (1.f - og) * acc[3][m][i];
                float cdn = fdot * cprev[e + u] + fg * cs[e + u] + idot * gg + ig * gdot;
                const float ca = act_f(act, cv);
                float hd = odot * ca + og * act_dy(act, ca) * cdn;
                if (!uok) { cdn = 0.f; hd = 0.f; }
                cs[e + u] = cdn;
                cprev[e + u] = cv;
                cd2[u] = cdn; hd2[u] = hd;
              }
              v0 = a0; v1 = a1; v2 = a2; v3 = a3; v4 = cd2; hv = hd2;
            }
            // unconditional: padded unit columns (c in [H, 112)) receive the zeros they must hold
            hnext[rr * LH + c] = f2bf(hv[0]);
            hnext[(rr + 1) * LH + c] = f2bf(hv[1]);
            if constexpr (TAPE) {
              pk[0][p] = pk2bf(v0[0], v0[1]); pk[1][p] = pk2bf(v1[0], v1[1]); pk[2][p] = pk2bf(v2[0], v2[1]);
              pk[3][p] = pk2bf(v3[0], v3[1]); pk[4][p] = pk2bf(v4[0], v4[1]);
            }
          }
          if constexpr (TAPE) {  // into this step's image; the data wave streams it out next step
            bf16_t* img = tsg + (t & 1) * FW4_STAGE + tape_off(0, wt32) + m * SLOT_HALF + lo8;
#pragma unroll
            for (int s = 0; s < TAPE_SLOTS; ++s)
              *reinterpret_cast<v2i*>(img + s * SLOT_ELEMS) = v2i{(int)pk[s][0], (int)pk[s][1]};
          }
        }
        if constexpr (TAN) {
#pragma unroll
          for (int s = 0; s < TAPE_SLOTS; ++s) tg[s] = tn[s];
        }
        xp.to_lds(xb + ((t + 1) & 1) * 32 * LX, trash, LX);  // (the last step's is unused)
        lds_barrier();  // step hand-off
      }
      __syncthreads();  // (C) the data wave has stored h_{T-1}
    }
  } else if (wave == 7) {
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      const int row0 = rb * 32;
      const rsrc_t rh = tile_rsrc(hs, row0, B, Tn, H);
      const rsrc_t rt = tape_rsrc(TAPE ? tape : nullptr, rb, nrb, Tn);
      const bool ton = !(dbg & 1);
      __syncthreads();  // (A)
      __syncthreads();  // (B)
      // stores only: with no load of its own this wave never waits on vmcnt (which retires loads
      // and stores in issue order), so the tape / h stream runs beside the recurrence
      for (int t = 0; t < Tn; ++t) {
        tile8_store_w<H>(hb + (t & 1) * 32 * LH, LH, rh, Tn, t - 1, t > 0 && !(dbg & 2), lane);
        if constexpr (TAPE)
          tape_image_store<H>(tsg + ((t + 1) & 1) * FW4_STAGE, rt, (dbg & 256) ? 0 : t - 1, t > 0 && ton, lane);
        lds_barrier();
      }
      tile8_store_w<H>(hb + (Tn & 1) * 32 * LH, LH, rh, Tn, Tn - 1, true, lane);
      if constexpr (TAPE)
        tape_image_store<H>(tsg + ((Tn - 1) & 1) * FW4_STAGE, rt, (dbg & 256) ? 0 : Tn - 1, ton, lane);
      __syncthreads();  // (C)
    }
  } else {
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
      __syncthreads();
      __syncthreads();
      for (int t = 0; t < Tn; ++t) lds_barrier();
      __syncthreads();
    }
  }
}

// ==========================================================================================
// host side
// ==========================================================================================
size_t lstm2_tape_elems(int B, int Tn) { return (size_t)((B + 31) / 32) * Tn * NW2 * TAPE_SLOTS * SLOT_ELEMS; }

static size_t tfwd2_smem(int H, int K) {
  const int KP = (K + 15) & ~15, LX = KP + 8, LH = ((H + 15) / 16) * 16 + 8;
  return (size_t)(4 * H * LX + 2 * 32 * LX + 2 * 32 * LH) * 2;
}
constexpr size_t LDS_MAX = 160 * 1024;

// Dynamic LDS above 64 KB needs the per-kernel attribute; set it once per kernel.
static void allow_big_lds(const void* kernel) {
  static std::mutex mu;
  static std::set<const void*> done;
  std::lock_guard<std::mutex> g(mu);
  if (done.insert(kernel).second)
    HFREP_CHECK_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX));
}

// persistent grid: one workgroup per CU (the kernels run at one or two waves per SIMD), each looping
// over row blocks so the weight fragments are loaded once per CU
static int persistent_grid(int B) {
  const int nrb = (B + 31) / 32, cus = device_cu_count();
  return nrb < cus ? nrb : cus;
}

static size_t fwd4_smem(int H, int K, bool tape) {  // generous: the 32-rounded extents (>= the tail-split ones)
  const int LX = fw4_stride((K + 31) & ~31), LH = fw4_stride(((H + 31) / 32) * 32);  // (>= fw4_stride of the split KP)
  return (size_t)(2 * 32 * LX + 2 * 32 * LH + (tape ? 2 * FW4_STAGE : 0) + 8) * 2;  // + trash
}

bool lstm2_supported(int H, int K) { return H == 100 && K >= 1 && K <= 128 && fwd4_smem(H, K, true) <= LDS_MAX; }

template <typename Kern, typename... Args>
static void launch(Kern k, int grid, int threads, size_t smem, hipStream_t s, Args... args) {
  allow_big_lds(reinterpret_cast<const void*>(k));
  hipLaunchKernelGGL(k, dim3(grid), dim3(threads), smem, s, args...);
}

// timing-only ablation mask of the forward kernel (HFREP_LSTM_DBG; 0 in every real run):
// 1 no tape store, 2 no h store, 4 no x load, 256 every step's tape stores to step 0's slots
// (L2-resident)
static int lstm_dbg() {
  static int d = -1;
  if (d < 0) {
    const char* e = getenv("HFREP_LSTM_DBG");
    d = e ? atoi(e) : 0;
  }
  return d;
}

// act (0 linear, 1 sigmoid, 2 tanh) and the input width K are template parameters: the cell
// activation switch and the x-tile index arithmetic would otherwise sit in the hottest loop.
// (the tangent forward is never instantiated for act = sigmoid: that instantiation was not bitwise
// reproducible at B = 32772 and launch_lstm2_tfwd routes act = 1 to lstm_tfwd2)
#define HFREP_FWD4_ACT(KXV, TP, TN, ...)                                                          \
  switch (act) {                                                                                 \
    case 0: launch(lstm_fwd4_kernel<100, 0, KXV, TP, TN>, __VA_ARGS__); break;                   \
    case 1:                                                                                      \
      if constexpr (!TN || HFREP_TFWD4_SIGMOID) launch(lstm_fwd4_kernel<100, 1, KXV, TP, TN>, __VA_ARGS__); \
      break;                                                                                     \
    default: launch(lstm_fwd4_kernel<100, 2, KXV, TP, TN>, __VA_ARGS__); break;                  \
  }
#define HFREP_FWD4_K(TP, TN, ...)                                                                \
  switch (K) {                                                                                   \
    case 32: HFREP_FWD4_ACT(32, TP, TN, __VA_ARGS__) break;                                      \
    case 35: HFREP_FWD4_ACT(35, TP, TN, __VA_ARGS__) break;                                      \
    case 36: HFREP_FWD4_ACT(36, TP, TN, __VA_ARGS__) break;                                      \
    case 100: HFREP_FWD4_ACT(100, TP, TN, __VA_ARGS__) break;                                    \
    default: HFREP_FWD4_ACT(0, TP, TN, __VA_ARGS__) break;                                       \
  }

void launch_lstm2_fwd(const void* x, const float* W, const float* b, const float* U, void* hs, void* tape, int B, int Tn,
                      int K, int H, int act, hipStream_t s) {
  const bf16_t* xp = (const bf16_t*)x;
  const int g = persistent_grid(B);
  const size_t sm = fwd4_smem(H, K, tape != nullptr);
  if (tape)
    HFREP_FWD4_K(true, false, g, 512, sm, s, xp, W, b, U, (const bf16_t*)nullptr, (bf16_t*)hs, (bf16_t*)tape, B, Tn, K, lstm_dbg())
  else
    HFREP_FWD4_K(false, false, g, 512, sm, s, xp, W, b, U, (const bf16_t*)nullptr, (bf16_t*)hs, (bf16_t*)nullptr, B, Tn, K,
                 lstm_dbg())
}

#define HFREP_TFWD2_K(...)                                                                       \
  switch (K) {                                                                                   \
    case 32: launch(lstm_tfwd2_kernel<100, 1, 32, 1>, __VA_ARGS__); break;                      \
    case 35: launch(lstm_tfwd2_kernel<100, 1, 35, 1>, __VA_ARGS__); break;                      \
    case 36: launch(lstm_tfwd2_kernel<100, 1, 36, 1>, __VA_ARGS__); break;                      \
    case 100: launch(lstm_tfwd2_kernel<100, 1, 100, 1>, __VA_ARGS__); break;                    \
    default: launch(lstm_tfwd2_kernel<100, 1, 0, 1>, __VA_ARGS__); break;                       \
  }

void launch_lstm2_tfwd(const void* xd, const float* W, const float* U, const void* tape, void* hds, void* ttape, int B,
                       int Tn, int K, int H, int act, hipStream_t s) {
  const bf16_t* xp = (const bf16_t*)xd;
  const int g = persistent_grid(B);
  if (act == 1 && !HFREP_TFWD4_SIGMOID) {
    // act = sigmoid: lstm_fwd4_kernel<.., TAN = true> differs run to run in rows 30 / 31 of a few row
    // blocks at B = 32772 (profiles/r03_race/README.md); the v2 tangent forward is bitwise there
    // (tests/test_kernels_gpu.py test_lstm2_tfwd_bitwise_large_batch).  Off the MTSS critic's path (tanh).
    HFREP_TFWD2_K(g, 256, tfwd2_smem(H, K), s, xp, W, U, (const bf16_t*)tape, (bf16_t*)hds, (bf16_t*)ttape, B, Tn, K)
    return;
  }
  HFREP_FWD4_K(true, true, g, 512, fwd4_smem(H, K, true), s, xp, W, (const float*)nullptr, U, (const bf16_t*)tape,
               (bf16_t*)hds, (bf16_t*)ttape, B, Tn, K, lstm_dbg())
}

// The bf16 BPTT is the tangent reverse v4 with its tangent stream compiled out (TG = false): 7 compute
// waves of 16 units on 16x16x32 MFMAs, two per SIMD, + 1 data wave.  It replaced lstm_bwd3 (4 recurrence
// waves of 32 units on 32x32x16, one per SIMD): 2-5 % faster per call at the bench shape, 9.06 -> 8.51 ms
// per B = 32 iteration -- with two compute waves per SIMD one wave's cell math runs under the other's
// MFMA chain (profiles/r05_bwd4).
#define HFREP_BWD4_ACT(DXV, GV, ...)                                                           \
  switch (act) {                                                                                 \
    case 0: launch(lstm_tbwd4_kernel<100, 0, DXV, GV, false>, __VA_ARGS__); break;               \
    case 1: launch(lstm_tbwd4_kernel<100, 1, DXV, GV, false>, __VA_ARGS__); break;               \
    default: launch(lstm_tbwd4_kernel<100, 2, DXV, GV, false>, __VA_ARGS__); break;              \
  }
#define HFREP_BWD4_LAUNCH(DXV, ...)                                                            \
  if (hw) HFREP_BWD4_ACT(DXV, true, __VA_ARGS__) else HFREP_BWD4_ACT(DXV, false, __VA_ARGS__)

void launch_lstm2_bwd(const void* dH, const void* tape, const float* U, void* dZ, const float* W, void* dX, int K,
                      int B, int Tn, int H, int act, hipStream_t s, const void* head_d, const float* hw) {
  const bf16_t* dh = (const bf16_t*)dH;
  const bf16_t* tp = (const bf16_t*)tape;
  const bf16_t* hd = (const bf16_t*)head_d;
  const bf16_t* nb = nullptr;
  bf16_t* nw = nullptr;
  const int g = persistent_grid(B);
  const size_t sm = Tb4Geo<100>::smem;
  if (dX)
    HFREP_BWD4_LAUNCH(true, g, 512, sm, s, dh, nb, tp, nb, U, (bf16_t*)dZ, nw, W, (bf16_t*)dX, nw, B, Tn, K, hd, nb, hw)
  else
    HFREP_BWD4_LAUNCH(false, g, 512, sm, s, dh, nb, tp, nb, U, (bf16_t*)dZ, nw, (const float*)nullptr, nw, nw, B, Tn, 0,
                      hd, nb, hw)
}

#define HFREP_TBWD4_ACT(DXV, GV, ...)                                                          \
  switch (act) {                                                                                 \
    case 0: launch(lstm_tbwd4_kernel<100, 0, DXV, GV>, __VA_ARGS__); break;                      \
    case 1: launch(lstm_tbwd4_kernel<100, 1, DXV, GV>, __VA_ARGS__); break;                      \
    default: launch(lstm_tbwd4_kernel<100, 2, DXV, GV>, __VA_ARGS__); break;                     \
  }
#define HFREP_TBWD4_LAUNCH(DXV, ...)                                                           \
  if (hw) HFREP_TBWD4_ACT(DXV, true, __VA_ARGS__) else HFREP_TBWD4_ACT(DXV, false, __VA_ARGS__)

void launch_lstm2_tbwd(const void* dH, const void* dHd, const void* tape, const void* ttape, const float* U, void* dZ,
                       void* dZd, const float* W, void* dX, void* dXd, int K, int B, int Tn, int H, int act,
                       hipStream_t s, const void* head_d, const void* head_dd, const float* hw) {
  const bf16_t* hd = (const bf16_t*)head_d;
  const bf16_t* hdd = (const bf16_t*)head_dd;
  const int g = persistent_grid(B);
  const size_t sm = Tb4Geo<100>::smem;
  // (DX + GEN -- generated head adjoint with the fused input gradient -- was parked in r01-r02 for
  // run-to-run drift: the cross-opcode MFMA SrcC hazard, fixed by xdl_switch; profiles/r03_race)
  if (dX)
    HFREP_TBWD4_LAUNCH(true, g, 512, sm, s, (const bf16_t*)dH, (const bf16_t*)dHd, (const bf16_t*)tape,
                       (const bf16_t*)ttape, U, (bf16_t*)dZ, (bf16_t*)dZd, W, (bf16_t*)dX, (bf16_t*)dXd, B, Tn, K, hd,
                       hdd, hw)
  else
    HFREP_TBWD4_LAUNCH(false, g, 512, sm, s, (const bf16_t*)dH, (const bf16_t*)dHd, (const bf16_t*)tape,
                       (const bf16_t*)ttape, U, (bf16_t*)dZ, (bf16_t*)dZd, (const float*)nullptr, (bf16_t*)nullptr,
                       (bf16_t*)nullptr, B, Tn, 0, hd, hdd, hw)
}

}  // namespace hfrep
