// One-shot peer-memory exchange for the SyncBN statistics.
//
// SyncBN issues one small blocking collective per BN layer and direction (49 all-gathers of
// (n, mean, M2) forward, 49 all-reduces of (sum g, sum g * xhat) backward per ResNet-50 step):
// 0.5-16 KB each, on the critical path, latency-bound.  Through RCCL each costs a collective
// launch plus its protocol round trips (17 us at world size 1 on MI355X).  Here every rank owns
// one "mailbox" buffer in its own HBM, mapped into every other rank's address space (HIP IPC,
// parallel/peer.py), and one single-workgroup kernel per exchange:
//   1. bumps the rank's device-side epoch e (so HIP-graph replays advance it too);
//   2. stores its n floats into slot [e & 1][rank] of EVERY rank's mailbox (remote stores over
//      xGMI; system-scope write-through stores, so nothing stays in this XCD's L2);
//   3. after every storing wave drained its stores and a system-scope release, sets flag[rank] = e
//      in every mailbox;
//   4. polls its own mailbox's flags until every rank's is >= e (system-scope loads, s_sleep
//      between polls), bounded by a wall-clock deadline (timeout_ms on the 100 MHz constant clock);
//   5. after a system-scope acquire, reads the world slots [e & 1][*] (system-scope loads) and
//      writes them out gathered ([world][n]) or summed in rank order ([n]; identical on every rank).
// A missed deadline FAILS LOUDLY instead of reading a stale slot: the kernel records err = 1, writes
// NaN into dst (so the statistics, the loss and every later step are visibly poisoned, never
// silently wrong), and every later exchange of this rank sees err != 0 and fails immediately the
// same way (no further waiting, no stores into the peers' mailboxes: a rank that lost the
// protocol must not overwrite slots a slower rank has yet to read).  The host raises on err at its
// next sync point (PeerExchange.check / peer.check_all, called by the training loop at every log
// interval and epoch end, and by bench.py's peer phase).
// Slots alternate by epoch parity: a rank can be at most one exchange ahead of the slowest (it
// needs everyone's flag for e before it starts e + 1), so its e + 1 stores never land in the
// parity a slower rank is still reading for e.
#include "common.cuh"
#include "launchers.h"

namespace dcp {

namespace {
constexpr int kPeerMaxWorld = 64;
constexpr uint64_t kWallHz = 100000000ull;  // s_memrealtime: 100 MHz constant clock on CDNA

__device__ __forceinline__ void poison(float* dst, int cnt, int tid) {
  for (int i = tid; i < cnt; i += blockDim.x) dst[i] = __builtin_nanf("");
}
}  // namespace

// mailbox layout (floats): [2 parities][world][slot] data, then flags (int) [world]
__global__ void __launch_bounds__(1024) peer_exchange_kernel(const float* __restrict__ src, int n,
                                                             float* __restrict__ dst, const int64_t* __restrict__ boxes,
                                                             int* __restrict__ epoch, int rank, int world, int slot,
                                                             int mode, int* __restrict__ err, int timeout_ms) {
  __shared__ int e_sh, bad_sh;
  const int tid = threadIdx.x;
  const int cnt = mode == 0 ? world * n : n;
  if (tid == 0) {
    const int e = *epoch + 1;
    *epoch = e;
    e_sh = e;
    bad_sh = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (bad_sh != 0) {  // an earlier exchange of this rank timed out: the protocol is lost, fail fast
    poison(dst, cnt, tid);
    return;
  }
  const int e = e_sh, par = e & 1;
  const size_t flags_off = (size_t)2 * world * slot;
  // 2. push this rank's data into every mailbox
  for (int r = 0; r < world; ++r) {
    float* box = reinterpret_cast<float*>(boxes[r]);
    float* dstslot = box + ((size_t)par * world + rank) * slot;
    for (int i = tid; i < n; i += blockDim.x)
      __hip_atomic_store(dstslot + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();
  // 3. publish: one lane per mailbox
  if (tid < world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* flags = reinterpret_cast<int*>(reinterpret_cast<float*>(boxes[tid]) + flags_off);
    __hip_atomic_store(flags + rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 4. wait for every rank's flag in this rank's own mailbox, up to the wall-clock deadline
  if (tid == 0) bad_sh = 0;
  __syncthreads();
  if (tid < world) {
    int* flags = reinterpret_cast<int*>(reinterpret_cast<float*>(boxes[rank]) + flags_off);
    const uint64_t t0 = wall_clock64();
    const uint64_t limit = (uint64_t)timeout_ms * (kWallHz / 1000ull);
    while (__hip_atomic_load(flags + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (wall_clock64() - t0 > limit) {
        atomicOr(err, 1);
        atomicOr(&bad_sh, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  if (bad_sh != 0) {  // a rank never published: poison instead of reading a stale parity slot
    poison(dst, cnt, tid);
    return;
  }
  // 5. gather / rank-ordered sum
  const float* mine = reinterpret_cast<const float*>(boxes[rank]) + (size_t)par * world * slot;
  if (mode == 0) {
    for (int i = tid; i < world * n; i += blockDim.x) {
      const int r = i / n, j = i - r * n;
      dst[i] = __hip_atomic_load(mine + (size_t)r * slot + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  } else {
    for (int j = tid; j < n; j += blockDim.x) {
      float acc = 0.f;
      for (int r = 0; r < world; ++r)
        acc += __hip_atomic_load(mine + (size_t)r * slot + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      dst[j] = acc;
    }
  }
}

bool launch_peer_exchange(const float* src, int n, float* dst, const int64_t* boxes, int* epoch, int rank, int world,
                          int slot, int mode, int* err, int timeout_ms, hipStream_t s) {
  if (world < 1 || world > kPeerMaxWorld || n > slot || rank < 0 || rank >= world || timeout_ms < 1) return false;
  hipLaunchKernelGGL(peer_exchange_kernel, dim3(1), dim3(1024), 0, s, src, n, dst, boxes, epoch, rank, world, slot,
                     mode, err, timeout_ms);
  return true;
}

}  // namespace dcp
