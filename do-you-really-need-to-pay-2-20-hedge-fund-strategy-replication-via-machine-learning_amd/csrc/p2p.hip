// One-shot all-reduce over peer-mapped device buffers (the optional custom xGMI
// collective next to RCCL).  The gradient buckets of this workload are ~0.5 MB: far below the
// ring-bandwidth regime, where RCCL's ring / tree pays 2 (W - 1) link latencies.  On the fully
// connected 8-GPU xGMI mesh every rank can instead read all peers' buckets at once, one link each:
// one flag hand-off and one pass.
//
// Each rank owns one buffer (fine-grained device memory, exported once through a HIP IPC handle and
// mapped by every peer):
//   [0, 4096)           control: epoch counter @0, finished-block counter @128, error word @256
//   [4096, 16384)       flags[src rank < 8][block < kP2PMaxBlocks]: src's block b staged epoch e
//   [16384, ...)        two data slots of `cap` floats (epoch parity)
// A call with epoch e (= the counter + 1) runs block b of every rank on chunk b of the bucket:
//   1. stage the local chunk into slot e & 1 of the OWN buffer; system-scope release;
//   2. write e into flags[rank][b] of EVERY rank's buffer (a remote store per peer);
//   3. wait (bounded) until flags[r][b] >= e for every r; system-scope acquire;
//   4. out = sum over r = 0 .. W-1 IN RANK ORDER of slot e & 1 of rank r (remote loads): every rank
//      computes the identical bits; then the scale (1 / W for an average).
// Slot parity makes one hand-off per call enough: a peer can only stage into slot e & 1 again at
// epoch e + 2, and its block b reaches that stage after its epoch e + 1 kernel saw all our epoch
// e + 1 flags, i.e. after our epoch e kernel -- and its reads of that slot -- completed.  The epoch
// lives in device memory (the last block of a call advances it), so the launch is hipGraph-safe.
// Failure is loud and sticky.  A wait is bounded by TIME (the constant-rate wall clock, `timeout_ticks`
// from HFREP_P2P_TIMEOUT_S): a block that gives up writes the error word of EVERY rank's buffer (the
// "poison"), and every waiting block of every rank polls its own error word, so the whole world
// leaves its waits within microseconds of the first give-up.  A block that did not complete the
// exchange writes NaN over its chunk of x (the runner's NaN guard then stops every rank at the next
// log record), the epoch counter is not advanced, and every later call on a poisoned buffer writes
// NaN at once without touching flags or peers.  The host reads the word asynchronously
// (P2PAllReduce.poll / GradSync.check_errors) and raises; there is no recovery -- the slot-parity
// argument above needs every rank in step, so a poisoned communicator is rebuilt, not reused.
#include "common.h"
#include "kernels.h"

#include <cstring>
#include <stdexcept>
#include <string>

namespace hfrep {

namespace {

__device__ inline void nan_fill(float* __restrict__ x, int64_t n, int64_t i0, int64_t i1, bool vec) {
  const float q = __builtin_nanf("");
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    if (vec) {
      reinterpret_cast<float4*>(x)[i] = make_float4(q, q, q, q);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (4 * i + k < n) x[4 * i + k] = q;
    }
  }
}

__global__ void __launch_bounds__(256) p2p_allreduce_kernel(float* __restrict__ x, int64_t n, P2PPeers peers,
                                                            int rank, int world, int64_t cap, float scale,
                                                            uint64_t timeout_ticks) {
  char* own = peers.base[rank];
  int* ctr = reinterpret_cast<int*>(own + kP2PCtr);
  int* done = reinterpret_cast<int*>(own + kP2PDone);
  int* err = reinterpret_cast<int*>(own + kP2PErr);
  __shared__ int s_epoch, s_dead;
  if (threadIdx.x == 0) {
    s_epoch = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    s_dead = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const int e = s_epoch;
  const int64_t slot = (int64_t)(e & 1) * cap;
  // this block's chunk, in float4 units (n4 rounds up; the last float4 may be partial)
  const int64_t n4 = (n + 3) >> 2, per = (n4 + gridDim.x - 1) / gridDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * per, i1 = i0 + per < n4 ? i0 + per : n4;
  const bool vec = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (s_dead) {  // poisoned by an earlier give-up (ours or a peer's): NaN, no flags, no waits
    nan_fill(x, n, i0, i1, vec);
    return;
  }

  // 1. stage
  float* mine = reinterpret_cast<float*>(own + kP2PData) + slot;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    if (vec) {
      reinterpret_cast<float4*>(mine)[i] = reinterpret_cast<const float4*>(x)[i];
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (4 * i + k < n) mine[4 * i + k] = x[4 * i + k];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the staged chunk before the flags
  __syncthreads();
  // 2. signal every rank (own included)
  if ((int)threadIdx.x < world) {
    int* fl = reinterpret_cast<int*>(peers.base[threadIdx.x] + kP2PFlags) + rank * kP2PMaxBlocks + blockIdx.x;
    __hip_atomic_store(fl, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every rank's chunk b, bounded by time; leave early when any rank has given up
  int ok = 1;
  if ((int)threadIdx.x < world) {
    const int* fl = reinterpret_cast<const int*>(own + kP2PFlags) + threadIdx.x * kP2PMaxBlocks + blockIdx.x;
    const uint64_t t0 = (uint64_t)wall_clock64();
    while (__hip_atomic_load(fl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
        ok = 0;
        break;
      }
      if ((uint64_t)wall_clock64() - t0 > timeout_ticks) {
        ok = 0;
        // poison every rank (own included): their waiting blocks see it at their next poll
        for (int r = 0; r < world; ++r)
          __hip_atomic_store(reinterpret_cast<int*>(peers.base[r] + kP2PErr), 1 + rank, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: peers' chunks after their flags
  // 4. reduce in rank order (or NaN: this chunk's exchange did not complete)
  if (ok) {
    for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
      if (vec) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int r = 0; r < world; ++r) {
          const float4 v = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(peers.base[r] + kP2PData) + slot)[i];
          s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
        reinterpret_cast<float4*>(x)[i] = s;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t j = 4 * i + k;
          if (j >= n) break;
          float s = 0.f;
          for (int r = 0; r < world; ++r) s += (reinterpret_cast<const float*>(peers.base[r] + kP2PData) + slot)[j];
          x[j] = s * scale;
        }
      }
    }
  } else {
    nan_fill(x, n, i0, i1, vec);
  }
  // epoch bookkeeping: the last block of the call advances the counter (the next call, later in
  // stream order, reads it) -- unless the call failed: a poisoned buffer keeps its epoch
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (int)gridDim.x - 1) {
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0)
        __hip_atomic_store(ctr, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

inline void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("hfrep p2p: ") + what + ": " + hipGetErrorString(e));
}

}  // namespace

size_t p2p_buffer_bytes(int64_t cap) { return (size_t)kP2PData + 2 * (size_t)cap * sizeof(float); }

void* p2p_alloc(int64_t cap, int device, bool* fine_grained) {
  int prev = 0;
  ck(hipGetDevice(&prev), "hipGetDevice");
  ck(hipSetDevice(device), "hipSetDevice");
  void* p = nullptr;
  const size_t bytes = p2p_buffer_bytes(cap);
  // fine-grained or nothing: the system-scope flag / data protocol above relies on it (coarse-grained
  // memory may serve a peer stale lines)
  ck(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained), "hipExtMallocWithFlags(fine-grained)");
  *fine_grained = true;
  ck(hipMemset(p, 0, bytes), "hipMemset");
  ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  ck(hipSetDevice(prev), "hipSetDevice");
  return p;
}

void p2p_free(void* p) { (void)hipFree(p); }

void p2p_ipc_handle(void* p, uint8_t out[64]) {
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "hipIpcMemHandle_t is 64 bytes");
  hipIpcMemHandle_t h;
  ck(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
  memcpy(out, &h, 64);
}

void* p2p_ipc_open(const uint8_t h[64], int device) {
  int prev = 0;
  ck(hipGetDevice(&prev), "hipGetDevice");
  ck(hipSetDevice(device), "hipSetDevice");
  hipIpcMemHandle_t hh;
  memcpy(&hh, h, 64);
  void* p = nullptr;
  ck(hipIpcOpenMemHandle(&p, hh, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  ck(hipSetDevice(prev), "hipSetDevice");
  return p;
}

void p2p_ipc_close(void* p) { (void)hipIpcCloseMemHandle(p); }

int p2p_read_error(void* own) {
  int e = 0;
  ck(hipMemcpy(&e, static_cast<char*>(own) + kP2PErr, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy");
  return e;
}

uint64_t p2p_timeout_ticks(double seconds, int device) {
  int khz = 0;
  ck(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device), "hipDeviceGetAttribute(WallClockRate)");
  if (khz <= 0) khz = 100000;  // gfx9's constant 100 MHz counter
  const double t = seconds * (double)khz * 1e3;
  return t <= 0 ? 1 : t >= 1.8e19 ? ~0ull : (uint64_t)t;
}

int p2p_blocks(int64_t n) {
  const int64_t b = (n + 4095) / 4096;  // >= 1024 float4 per block
  return (int)(b < 1 ? 1 : b > kP2PMaxBlocks ? kP2PMaxBlocks : b);
}

void launch_p2p_allreduce(float* x, int64_t n, const P2PPeers& peers, int rank, int world, int64_t cap, float scale,
                          uint64_t timeout_ticks, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(p2p_allreduce_kernel, dim3(p2p_blocks(n)), dim3(256), 0, s, x, n, peers, rank, world, cap, scale,
                     timeout_ticks);
}

}  // namespace hfrep
