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
//    GP's reverse pass) are stored in a BLOCKED layout [rowblock][t][wave][slot][lane][16] that
//    matches the accumulator layout: each lane moves its 16 values with two 16-byte accesses;
//  * row-major activations (h, dH, dZ) go through the LDS tile that the recurrence needs anyway
//    and are streamed to/from HBM with coalesced 8-byte accesses by the whole workgroup.
//
// Contracts are identical to ops/reference.py (lstm_seq_*), with zx = x W + b folded in.
#include "common.h"
#include "mfma.h"
#include "kernels.h"

namespace hfrep {

namespace {

constexpr int NW2 = 4;       // waves per workgroup: 4 x 32 units covers H <= 128
constexpr int TAPE_SLOTS = 5;  // 4 gates (or 4 tangent pre-activations) + cell (or cell tangent)
constexpr int SLOT_ELEMS = 64 * 16;

__device__ __forceinline__ size_t tape_base(int rb, int t, int Tn, int w) {
  return (((size_t)rb * Tn + t) * NW2 + w) * TAPE_SLOTS * SLOT_ELEMS;
}

__device__ __forceinline__ uint32_t pk2(float lo, float hi) { return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16); }
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
__device__ __forceinline__ Slot16 ld_slot(const bf16_t* p) {
  Slot16 s;
  s.a = reinterpret_cast<const uint4*>(p)[0];
  s.b = reinterpret_cast<const uint4*>(p)[1];
  return s;
}
__device__ __forceinline__ void st_slot(bf16_t* p, const uint32_t (&v)[8]) {
  reinterpret_cast<uint4*>(p)[0] = make_uint4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<uint4*>(p)[1] = make_uint4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void put4(uint32_t (&v)[4], int i, float x) {
  if (i & 1) v[i >> 1] |= ((uint32_t)f2bf(x) << 16);
  else v[i >> 1] = (uint32_t)f2bf(x);
}

// stage W^T (K x G fp32, row-major) into LDS as bf16 [G][LX], zero-padded in k
__device__ __forceinline__ void stage_wt(bf16_t* Wt, const float* __restrict__ W, int K, int G, int LX) {
  for (int e = threadIdx.x; e < G * LX; e += blockDim.x) {
    const int k = e / G, n = e % G;  // consecutive threads read consecutive n (coalesced)
    if (k < LX) Wt[n * LX + k] = f2bf(k < K ? W[(size_t)k * G + n] : 0.f);
  }
}

// x tile (32 rows x K, time t) -> registers (up to 16 bf16 per thread)
struct XPref {
  uint32_t v[8];  // 16 bf16, two per register
};
__device__ __forceinline__ void x_load(XPref& p, const bf16_t* __restrict__ x, int row0, int B, int Tn, int t, int K) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int e = threadIdx.x + 256 * j;
    const int r = e / K, k = e - r * K;
    const int row = row0 + r;
    const uint32_t v = (r < 32 && row < B) ? (uint32_t)x[((size_t)row * Tn + t) * K + k] : 0u;
    if (j & 1) p.v[j >> 1] |= v << 16;
    else p.v[j >> 1] = v;
  }
}
__device__ __forceinline__ void x_store_lds(const XPref& p, bf16_t* xb, int K, int LX) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int e = threadIdx.x + 256 * j;
    const int r = e / K, k = e - r * K;
    if (r < 32) xb[r * LX + k] = (bf16_t)((j & 1) ? (p.v[j >> 1] >> 16) : (p.v[j >> 1] & 0xffffu));
  }
}

// row-major [32 x H] tile <-> HBM (B,T,H) with 8-byte chunks (H % 4 == 0)
template <int H>
__device__ __forceinline__ void tile_to_hbm(const bf16_t* buf, int LD, bf16_t* __restrict__ dst, int row0, int B, int Tn,
                                            int t, int width) {
  const int cpr = width / 4;
  for (int e = threadIdx.x; e < 32 * cpr; e += 256) {
    const int r = e / cpr, c = e - r * cpr;
    const int row = row0 + r;
    if (row < B)
      *reinterpret_cast<uint2*>(dst + ((size_t)row * Tn + t) * width + 4 * c) =
          *reinterpret_cast<const uint2*>(buf + r * LD + 4 * c);
  }
}
template <int H>
__device__ __forceinline__ void tile_from_hbm(bf16_t* buf, int LD, const bf16_t* __restrict__ src, int row0, int B,
                                              int Tn, int t, int width) {
  const int cpr = width / 4;
  for (int e = threadIdx.x; e < 32 * cpr; e += 256) {
    const int r = e / cpr, c = e - r * cpr;
    const int row = row0 + r;
    uint2 v = make_uint2(0, 0);
    if (row < B) v = *reinterpret_cast<const uint2*>(src + ((size_t)row * Tn + t) * width + 4 * c);
    *reinterpret_cast<uint2*>(buf + r * LD + 4 * c) = v;
  }
}

}  // namespace

// ==========================================================================================
// forward (+ optional tape):  z_t = x_t W + b + h_{t-1} U
// ==========================================================================================
template <int H, int ACT>
__global__ void __launch_bounds__(256)
lstm_fwd2_kernel(const bf16_t* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                 const float* __restrict__ U, bf16_t* __restrict__ hs, bf16_t* __restrict__ tape, int B, int Tn, int K,
                 int act_rt) {
  constexpr int act = ACT;
  (void)act_rt;
  using P = MF<bf16_t>;
  constexpr int G = 4 * H, NKH = (H + 15) / 16, LH = NKH * 16 + 8, KPADH = NKH * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int KP = (K + 15) & ~15, LX = KP + 8, NKX = KP / 16;
  bf16_t* Wt = reinterpret_cast<bf16_t*>(smem);
  bf16_t* xb = Wt + G * LX;
  bf16_t* hb = xb + 2 * 32 * LX;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int uc = uok ? u : H - 1;
  const int nrb = (B + 31) / 32;

  // per-workgroup prologue, amortised over every row block this persistent workgroup owns
  stage_wt(Wt, W, K, G, LX);
  for (int i = threadIdx.x; i < 2 * 32 * LX; i += 256) xb[i] = 0;
  typename P::frag ub[4][NKH];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int ks = 0; ks < NKH; ++ks)
      ub[q][ks] = P::make([&](int k) { return (uok && k < H) ? U[k * G + q * H + u] : 0.f; }, ks, lane);
  float bq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bq[q] = (uok && bias) ? bias[q * H + u] : 0.f;

  for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
  const int row0 = rb * 32;
  for (int i = threadIdx.x; i < 2 * 32 * LH; i += 256) hb[i] = 0;
  float c[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  XPref pf;
  __syncthreads();
  x_load(pf, x, row0, B, Tn, 0, K);
  x_store_lds(pf, xb, K, LX);
  __syncthreads();

  for (int t = 0; t < Tn; ++t) {
    const bf16_t* xcur = xb + (t & 1) * 32 * LX;
    const bf16_t* hcur = hb + (t & 1) * 32 * LH;
    bf16_t* hnext = hb + ((t + 1) & 1) * 32 * LH;
    if (t > 0) tile_to_hbm<H>(hcur, LH, hs, row0, B, Tn, t - 1, H);
    if (t + 1 < Tn) x_load(pf, x, row0, B, Tn, t + 1, K);
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
    for (int half = 0; half < 2; ++half) {  // two halves of 8 rows: 20 packing registers, not 40
      uint32_t pk[TAPE_SLOTS][4];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = half * 8 + i;
        const int rr = acc32_row(r, lane);
        const float ig = sigmoidf_(acc[0][r] + bq[0]), fg = sigmoidf_(acc[1][r] + bq[1]);
        const float gg = act_f(act, acc[2][r] + bq[2]), og = sigmoidf_(acc[3][r] + bq[3]);
        float cn = fg * c[r] + ig * gg;
        float h = og * act_f(act, cn);
        if (!uok) { cn = 0.f; h = 0.f; }
        c[r] = cn;
        if (u < KPADH) hnext[rr * LH + u] = f2bf(h);
        put4(pk[0], i, ig); put4(pk[1], i, fg); put4(pk[2], i, gg); put4(pk[3], i, og); put4(pk[4], i, cn);
      }
      if (tape) {
        bf16_t* tp = tape + tape_base(rb, t, Tn, w) + lane * 16 + half * 8;
#pragma unroll
        for (int s = 0; s < TAPE_SLOTS; ++s)
          *reinterpret_cast<uint4*>(tp + s * SLOT_ELEMS) = make_uint4(pk[s][0], pk[s][1], pk[s][2], pk[s][3]);
      }
    }
    if (t + 1 < Tn) x_store_lds(pf, xb + ((t + 1) & 1) * 32 * LX, K, LX);
    __syncthreads();
  }
  tile_to_hbm<H>(hb + (Tn & 1) * 32 * LH, LH, hs, row0, B, Tn, Tn - 1, H);
  __syncthreads();  // LDS is re-initialised for the next row block
  }
}

// ==========================================================================================
// tangent forward at the taped primal point: zdot_t = xdot_t W + hdot_{t-1} U
// ==========================================================================================
template <int H, int ACT>
__global__ void __launch_bounds__(256)
lstm_tfwd2_kernel(const bf16_t* __restrict__ xd, const float* __restrict__ W, const float* __restrict__ U,
                  const bf16_t* __restrict__ tape, bf16_t* __restrict__ hds, bf16_t* __restrict__ ttape, int B, int Tn,
                  int K, int act_rt) {
  constexpr int act = ACT;
  (void)act_rt;
  using P = MF<bf16_t>;
  constexpr int G = 4 * H, NKH = (H + 15) / 16, LH = NKH * 16 + 8, KPADH = NKH * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int KP = (K + 15) & ~15, LX = KP + 8, NKX = KP / 16;
  bf16_t* Wt = reinterpret_cast<bf16_t*>(smem);
  bf16_t* xb = Wt + G * LX;
  bf16_t* hb = xb + 2 * 32 * LX;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int uc = uok ? u : H - 1;
  const int nrb = (B + 31) / 32;

  stage_wt(Wt, W, K, G, LX);
  for (int i = threadIdx.x; i < 2 * 32 * LX; i += 256) xb[i] = 0;
  typename P::frag ub[4][NKH];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int ks = 0; ks < NKH; ++ks)
      ub[q][ks] = P::make([&](int k) { return (uok && k < H) ? U[k * G + q * H + u] : 0.f; }, ks, lane);

  for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
  const int row0 = rb * 32;
  for (int i = threadIdx.x; i < 2 * 32 * LH; i += 256) hb[i] = 0;
  float cd[16], cprev[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) { cd[r] = 0.f; cprev[r] = 0.f; }
  XPref pf;
  __syncthreads();
  x_load(pf, xd, row0, B, Tn, 0, K);
  x_store_lds(pf, xb, K, LX);
  // primal tape of step 0 (gates + cell)
  Slot16 tg[TAPE_SLOTS];
  {
    const bf16_t* tp = tape + tape_base(rb, 0, Tn, w) + lane * 16;
#pragma unroll
    for (int s = 0; s < TAPE_SLOTS; ++s) tg[s] = ld_slot(tp + s * SLOT_ELEMS);
  }
  __syncthreads();

  for (int t = 0; t < Tn; ++t) {
    const bf16_t* xcur = xb + (t & 1) * 32 * LX;
    const bf16_t* hcur = hb + (t & 1) * 32 * LH;
    bf16_t* hnext = hb + ((t + 1) & 1) * 32 * LH;
    if (t > 0) tile_to_hbm<H>(hcur, LH, hds, row0, B, Tn, t - 1, H);
    Slot16 tn[TAPE_SLOTS];
    if (t + 1 < Tn) {
      x_load(pf, xd, row0, B, Tn, t + 1, K);
      const bf16_t* tp = tape + tape_base(rb, t + 1, Tn, w) + lane * 16;
#pragma unroll
      for (int s = 0; s < TAPE_SLOTS; ++s) tn[s] = ld_slot(tp + s * SLOT_ELEMS);
    }
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
      bf16_t* tp = ttape + tape_base(rb, t, Tn, w) + lane * 16 + half * 8;
#pragma unroll
      for (int s = 0; s < TAPE_SLOTS; ++s)
        *reinterpret_cast<uint4*>(tp + s * SLOT_ELEMS) = make_uint4(pk[s][0], pk[s][1], pk[s][2], pk[s][3]);
    }
    if (t + 1 < Tn) {
      x_store_lds(pf, xb + ((t + 1) & 1) * 32 * LX, K, LX);
#pragma unroll
      for (int s = 0; s < TAPE_SLOTS; ++s) tg[s] = tn[s];
    }
    __syncthreads();
  }
  tile_to_hbm<H>(hb + (Tn & 1) * 32 * LH, LH, hds, row0, B, Tn, Tn - 1, H);
  __syncthreads();
  }
}

// ==========================================================================================
// BPTT: dZ (B,T,4H) row-major from dH (B,T,H) and the tape
// ==========================================================================================
template <int H, int ACT>
__global__ void __launch_bounds__(256)
lstm_bwd2_kernel(const bf16_t* __restrict__ dH, const bf16_t* __restrict__ tape, const float* __restrict__ U,
                 bf16_t* __restrict__ dZ, int B, int Tn, int act_rt) {
  constexpr int act = ACT;
  (void)act_rt;
  using P = MF<bf16_t>;
  constexpr int G = 4 * H, NKG = (G + 15) / 16, LG = NKG * 16 + 8, NKH = (H + 15) / 16, LH = NKH * 16 + 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* zb = reinterpret_cast<bf16_t*>(smem);  // [2][32][LG]
  bf16_t* dhb = zb + 2 * 32 * LG;                 // [2][32][LH]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int nrb = (B + 31) / 32;

  typename P::frag ut[NKG];
#pragma unroll
  for (int ks = 0; ks < NKG; ++ks)
    ut[ks] = P::make([&](int k) { return (uok && k < G) ? U[u * G + k] : 0.f; }, ks, lane);
  for (int i = threadIdx.x; i < 2 * 32 * LG; i += 256) zb[i] = 0;

  for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
  const int row0 = rb * 32;
  float dc[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) dc[r] = 0.f;
  __syncthreads();
  tile_from_hbm<H>(dhb + ((Tn - 1) & 1) * 32 * LH, LH, dH, row0, B, Tn, Tn - 1, H);
  Slot16 tg[4], cc, cp;
  {
    const bf16_t* tp = tape + tape_base(rb, Tn - 1, Tn, w) + lane * 16;
#pragma unroll
    for (int s = 0; s < 4; ++s) tg[s] = ld_slot(tp + s * SLOT_ELEMS);
    cc = ld_slot(tp + 4 * SLOT_ELEMS);
    cp.a = make_uint4(0, 0, 0, 0); cp.b = cp.a;
    if (Tn > 1) cp = ld_slot(tape + tape_base(rb, Tn - 2, Tn, w) + lane * 16 + 4 * SLOT_ELEMS);
  }
  __syncthreads();

  for (int t = Tn - 1; t >= 0; --t) {
    const bf16_t* zprev = zb + ((t + 1) & 1) * 32 * LG;  // dz_{t+1}
    bf16_t* zcur = zb + (t & 1) * 32 * LG;               // dz_t
    const bf16_t* dhcur = dhb + (t & 1) * 32 * LH;
    if (t < Tn - 1) tile_to_hbm<H>(zprev, LG, dZ, row0, B, Tn, t + 1, G);
    // prefetch the next (t-1) step: tape gates(t-1), cell(t-2), dH(t-1)
    Slot16 ng[4], ncp;
    uint2 ndh[4];
    if (t > 0) {
      const bf16_t* tp = tape + tape_base(rb, t - 1, Tn, w) + lane * 16;
#pragma unroll
      for (int s = 0; s < 4; ++s) ng[s] = ld_slot(tp + s * SLOT_ELEMS);
      ncp.a = make_uint4(0, 0, 0, 0); ncp.b = ncp.a;
      if (t > 1) ncp = ld_slot(tape + tape_base(rb, t - 2, Tn, w) + lane * 16 + 4 * SLOT_ELEMS);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = threadIdx.x + 256 * j;
        const int r = e / (H / 4), c4 = e - r * (H / 4);
        const int row = row0 + r;
        ndh[j] = make_uint2(0, 0);
        if (r < 32 && row < B) ndh[j] = *reinterpret_cast<const uint2*>(dH + ((size_t)row * Tn + (t - 1)) * H + 4 * c4);
      }
    }
    f32x16 acc = zero16();
    if (t < Tn - 1) {
      const bf16_t* arow = zprev + (lane & 31) * LG;
#pragma unroll
      for (int ks = 0; ks < NKG; ++ks) acc = P::mma(P::lda(arow, ks, lane), ut[ks], acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = acc32_row(r, lane);
      const float ig = tg[0].get(r), fg = tg[1].get(r), gg = tg[2].get(r), og = tg[3].get(r);
      const float c = cc.get(r), cpv = cp.get(r);
      const float dht = (uok ? bf2f(dhcur[rr * LH + u]) : 0.f) + acc[r];
      const float ca = act_f(act, c);
      const float dov = dht * ca;
      const float dct = dc[r] + dht * og * act_dy(act, ca);
      dc[r] = uok ? dct * fg : 0.f;
      float z0 = dct * gg * ig * (1.f - ig);
      float z1 = dct * cpv * fg * (1.f - fg);
      float z2 = dct * ig * act_dy(act, gg);
      float z3 = dov * og * (1.f - og);
      if (uok) {
        bf16_t* zr = zcur + rr * LG + u;
        zr[0] = f2bf(z0); zr[H] = f2bf(z1); zr[2 * H] = f2bf(z2); zr[3 * H] = f2bf(z3);
      }
    }
    if (t > 0) {
      bf16_t* dnext = dhb + ((t - 1) & 1) * 32 * LH;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = threadIdx.x + 256 * j;
        const int r = e / (H / 4), c4 = e - r * (H / 4);
        if (r < 32) *reinterpret_cast<uint2*>(dnext + r * LH + 4 * c4) = ndh[j];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) tg[s] = ng[s];
      cc = cp;
      cp = ncp;
    }
    __syncthreads();
  }
  tile_to_hbm<H>(zb, LG, dZ, row0, B, Tn, 0, G);
  __syncthreads();
  }
}

// ==========================================================================================
// reverse of the tangent system: (dZ, dZd) from (dH?, dHd), primal tape and tangent tape
// ==========================================================================================
template <int H, int ACT>
__global__ void __launch_bounds__(256)
lstm_tbwd2_kernel(const bf16_t* __restrict__ dH, const bf16_t* __restrict__ dHd, const bf16_t* __restrict__ tape,
                  const bf16_t* __restrict__ ttape, const float* __restrict__ U, bf16_t* __restrict__ dZ,
                  bf16_t* __restrict__ dZd, int B, int Tn, int act_rt) {
  constexpr int act = ACT;
  (void)act_rt;
  using P = MF<bf16_t>;
  constexpr int G = 4 * H, NKG = (G + 15) / 16, LG = NKG * 16 + 8, NKH = (H + 15) / 16, LH = NKH * 16 + 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* zb = reinterpret_cast<bf16_t*>(smem);  // [2][32][LG]
  bf16_t* zdb = zb + 2 * 32 * LG;                 // [2][32][LG]
  bf16_t* dhb = zdb + 2 * 32 * LG;                // [2][32][LH]  (dH)
  bf16_t* dhdb = dhb + 2 * 32 * LH;               // [2][32][LH]  (dHdot)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int nrb = (B + 31) / 32;

  typename P::frag ut[NKG];
#pragma unroll
  for (int ks = 0; ks < NKG; ++ks)
    ut[ks] = P::make([&](int k) { return (uok && k < G) ? U[u * G + k] : 0.f; }, ks, lane);
  for (int i = threadIdx.x; i < 2 * 32 * LG; i += 256) { zb[i] = 0; zdb[i] = 0; }
  for (int i = threadIdx.x; i < 2 * 32 * LH; i += 256) dhb[i] = 0;

  for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
  const int row0 = rb * 32;
  float ac[16], acd[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) { ac[r] = 0.f; acd[r] = 0.f; }
  __syncthreads();
  if (dH) tile_from_hbm<H>(dhb + ((Tn - 1) & 1) * 32 * LH, LH, dH, row0, B, Tn, Tn - 1, H);
  tile_from_hbm<H>(dhdb + ((Tn - 1) & 1) * 32 * LH, LH, dHd, row0, B, Tn, Tn - 1, H);
  Slot16 cc, cdc;  // c_t and cdot_t carried (loaded at the previous iteration as "prev")
  {
    const size_t b = tape_base(rb, Tn - 1, Tn, w) + lane * 16 + 4 * SLOT_ELEMS;
    cc = ld_slot(tape + b);
    cdc = ld_slot(ttape + b);
  }
  __syncthreads();

  for (int t = Tn - 1; t >= 0; --t) {
    const int cb = t & 1, nb = (t + 1) & 1;
    if (t < Tn - 1) {
      tile_to_hbm<H>(zb + nb * 32 * LG, LG, dZ, row0, B, Tn, t + 1, G);
      tile_to_hbm<H>(zdb + nb * 32 * LG, LG, dZd, row0, B, Tn, t + 1, G);
    }
    // this step's tapes
    Slot16 tg[4], zd[4], cp, cdp;
    {
      const bf16_t* tp = tape + tape_base(rb, t, Tn, w) + lane * 16;
      const bf16_t* tq = ttape + tape_base(rb, t, Tn, w) + lane * 16;
#pragma unroll
      for (int s = 0; s < 4; ++s) { tg[s] = ld_slot(tp + s * SLOT_ELEMS); zd[s] = ld_slot(tq + s * SLOT_ELEMS); }
      cp.a = make_uint4(0, 0, 0, 0); cp.b = cp.a; cdp = cp;
      if (t > 0) {
        const size_t b = tape_base(rb, t - 1, Tn, w) + lane * 16 + 4 * SLOT_ELEMS;
        cp = ld_slot(tape + b);
        cdp = ld_slot(ttape + b);
      }
    }
    f32x16 ah = zero16(), ahd = zero16();
    if (t < Tn - 1) {
      const bf16_t* arow = zb + nb * 32 * LG + (lane & 31) * LG;
      const bf16_t* drow = zdb + nb * 32 * LG + (lane & 31) * LG;
#pragma unroll
      for (int ks = 0; ks < NKG; ++ks) {
        ah = P::mma(P::lda(arow, ks, lane), ut[ks], ah);
        ahd = P::mma(P::lda(drow, ks, lane), ut[ks], ahd);
      }
    }
    const bf16_t* dh_t = dhb + cb * 32 * LH;
    const bf16_t* dhd_t = dhdb + cb * 32 * LH;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = acc32_row(r, lane);
      const float ig = tg[0].get(r), fg = tg[1].get(r), gg = tg[2].get(r), og = tg[3].get(r);
      const float c = cc.get(r), cpv = cp.get(r), cd = cdc.get(r), cdpv = cdp.get(r);
      const float zdi = zd[0].get(r), zdf = zd[1].get(r), zdg = zd[2].get(r), zdo = zd[3].get(r);
      const float si = ig * (1.f - ig), sf = fg * (1.f - fg), so = og * (1.f - og);
      const float sg = act_dy(act, gg);
      const float idot = si * zdi, fdot = sf * zdf, gdot = sg * zdg, odot = so * zdo;
      const float ca = act_f(act, c);
      const float e1 = act_dy(act, ca), e2 = act_d2y(act, ca);
      const float a_h = (uok ? bf2f(dh_t[rr * LH + u]) : 0.f) + ah[r];
      const float a_hd = (uok ? bf2f(dhd_t[rr * LH + u]) : 0.f) + ahd[r];
      const float a_od = a_hd * ca;
      const float a_o = a_h * ca + a_hd * e1 * cd;
      const float a_cd = acd[r] + a_hd * og * e1;
      const float a_c = ac[r] + a_h * og * e1 + a_hd * (odot * e1 + og * e2 * cd);
      const float a_fd = a_cd * cpv, a_id = a_cd * gg, a_gd = a_cd * ig;
      const float a_f = a_c * cpv + a_cd * cdpv;
      const float a_i = a_c * gg + a_cd * gdot;
      const float a_g = a_c * ig + a_cd * idot;
      ac[r] = uok ? a_c * fg + a_cd * fdot : 0.f;
      acd[r] = uok ? a_cd * fg : 0.f;
      const float s2i = si * (1.f - 2.f * ig), s2f = sf * (1.f - 2.f * fg), s2o = so * (1.f - 2.f * og);
      const float s2g = act_d2y(act, gg);
      if (uok) {
        bf16_t* zr = zb + cb * 32 * LG + rr * LG + u;
        bf16_t* dr = zdb + cb * 32 * LG + rr * LG + u;
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
    if (t > 0) {
      if (dH) tile_from_hbm<H>(dhb + nb * 32 * LH, LH, dH, row0, B, Tn, t - 1, H);
      tile_from_hbm<H>(dhdb + nb * 32 * LH, LH, dHd, row0, B, Tn, t - 1, H);
      cc = cp;
      cdc = cdp;
    }
    __syncthreads();
  }
  tile_to_hbm<H>(zb, LG, dZ, row0, B, Tn, 0, G);
  tile_to_hbm<H>(zdb, LG, dZd, row0, B, Tn, 0, G);
  __syncthreads();
  }
}

// ==========================================================================================
// host side
// ==========================================================================================
size_t lstm2_tape_elems(int B, int Tn) { return (size_t)((B + 31) / 32) * Tn * NW2 * TAPE_SLOTS * SLOT_ELEMS; }

static size_t fwd_smem(int H, int K) {
  const int KP = (K + 15) & ~15, LX = KP + 8, LH = ((H + 15) / 16) * 16 + 8;
  return (size_t)(4 * H * LX + 2 * 32 * LX + 2 * 32 * LH) * 2;
}
static size_t bwd_smem(int H) {
  const int LG = ((4 * H + 15) / 16) * 16 + 8, LH = ((H + 15) / 16) * 16 + 8;
  return (size_t)(2 * 32 * LG + 2 * 32 * LH) * 2;
}
static size_t tbwd_smem(int H) {
  const int LG = ((4 * H + 15) / 16) * 16 + 8, LH = ((H + 15) / 16) * 16 + 8;
  return (size_t)(4 * 32 * LG + 4 * 32 * LH) * 2;
}

// Dynamic LDS above 64 KB needs the per-kernel attribute; set it once per instantiation.
template <typename K>
static void allow_big_lds(K kernel) {
  static bool done = false;
  if (!done) {
    HFREP_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    done = true;
  }
}

// persistent grid: one workgroup per CU (the kernels run at one wave per SIMD), each looping over
// row blocks so the W^T staging and the register-resident U fragments are paid once per CU
static int persistent_grid(int B) {
  const int nrb = (B + 31) / 32, cus = device_cu_count();
  return nrb < cus ? nrb : cus;
}

bool lstm2_supported(int H, int K) { return H == 100 && K >= 1 && K <= 128 && fwd_smem(H, K) <= 160 * 1024; }

// act is a template parameter (0 linear, 1 sigmoid, 2 tanh): the cell-activation switch would
// otherwise cost registers and instructions in the hottest loop
#define HFREP_ACT_DISPATCH(act, KERNEL, ...)                                 \
  switch (act) {                                                             \
    case 0: { auto k = KERNEL<100, 0>; allow_big_lds(k); hipLaunchKernelGGL(k, __VA_ARGS__); break; } \
    case 1: { auto k = KERNEL<100, 1>; allow_big_lds(k); hipLaunchKernelGGL(k, __VA_ARGS__); break; } \
    default: { auto k = KERNEL<100, 2>; allow_big_lds(k); hipLaunchKernelGGL(k, __VA_ARGS__); break; } \
  }

void launch_lstm2_fwd(const void* x, const float* W, const float* b, const float* U, void* hs, void* tape, int B, int Tn,
                      int K, int H, int act, hipStream_t s) {
  HFREP_ACT_DISPATCH(act, lstm_fwd2_kernel, dim3(persistent_grid(B)), dim3(256), fwd_smem(H, K), s, (const bf16_t*)x, W, b,
                     U, (bf16_t*)hs, (bf16_t*)tape, B, Tn, K, act)
}
void launch_lstm2_tfwd(const void* xd, const float* W, const float* U, const void* tape, void* hds, void* ttape, int B,
                       int Tn, int K, int H, int act, hipStream_t s) {
  HFREP_ACT_DISPATCH(act, lstm_tfwd2_kernel, dim3(persistent_grid(B)), dim3(256), fwd_smem(H, K), s, (const bf16_t*)xd, W,
                     U, (const bf16_t*)tape, (bf16_t*)hds, (bf16_t*)ttape, B, Tn, K, act)
}
void launch_lstm2_bwd(const void* dH, const void* tape, const float* U, void* dZ, int B, int Tn, int H, int act,
                      hipStream_t s) {
  HFREP_ACT_DISPATCH(act, lstm_bwd2_kernel, dim3(persistent_grid(B)), dim3(256), bwd_smem(H), s, (const bf16_t*)dH,
                     (const bf16_t*)tape, U, (bf16_t*)dZ, B, Tn, act)
}
void launch_lstm2_tbwd(const void* dH, const void* dHd, const void* tape, const void* ttape, const float* U, void* dZ,
                       void* dZd, int B, int Tn, int H, int act, hipStream_t s) {
  HFREP_ACT_DISPATCH(act, lstm_tbwd2_kernel, dim3(persistent_grid(B)), dim3(256), tbwd_smem(H), s, (const bf16_t*)dH,
                     (const bf16_t*)dHd, (const bf16_t*)tape, (const bf16_t*)ttape, U, (bf16_t*)dZ, (bf16_t*)dZd, B,
                     Tn, act)
}

}  // namespace hfrep
