// lhpc_dist.hip — multi-GPU SpMV and stencil behind the C ABI: one process
// per GPU, one RCCL communicator (over xGMI) and one communication stream per
// process (SURVEY §8b "one stream and one RCCL comm per device", §8e).
//
// The reference has no multi-device code; its only overlap idiom
// is the chunked copy/compute stream pipeline of
// lib/gpu/transfer_overlap_testsuite/src/cuda_tut_transfer_overlap.cu:41-142,
// which the chunk loop of lhpc_dist_spmv follows with a collective in place
// of the copy.
//
//   SpMV   rows cut into nranks·K nnz-balanced blocks (lhpc_csr_partition_rows
//          with nranks·K parts); block b = k·nranks + r is rank r's chunk k.
//          A rank stages x once (the XTILE tile gather of a row-range plan
//          over its K blocks), then for k = 0..K−1 reduces chunk k straight
//          into its rows of the full y and hands chunk k to the comm stream,
//          where one in-place ncclAllGather (equal-size blocks) or a group of
//          nranks in-place ncclBroadcast (root r sends block k·nranks + r;
//          exact slices, no padding) fills every rank's y while the compute
//          stream reduces chunk k+1.  y is then the next x on every rank.
//          Direct peer exchange (SURVEY §8e "Optimisation"): with registered
//          y windows (lhpc_dist_p2p_export/_import: IPC handles of every
//          rank's y; up to four, so a ping-pong pair works), chunk k's block
//          is pushed by one kernel straight into every peer's y over xGMI
//          instead of the collectives; per call a READY flag (this rank's y
//          may be overwritten) and a DONE flag (this rank's pushes have
//          landed) go to every peer, and the comm stream waits for all
//          peers' flags with a bounded spin.  Needs no RCCL communicator
//          (lhpc_dist_comm_create_local).  The exchange is a plan option
//          (lhpc_options.dist_exchange: automatic = peer stores when y is a
//          window).  Both exchanges issue the transfers of one host
//          schedule (lhpc_dist_exchange_schedule), which the CPU tests run.
//   stencil z-slabs with one halo plane per side: ncclSend/ncclRecv to the
//          z neighbours on the comm stream while the interior planes are
//          computed; the two boundary planes after the exchange.
// Status: RCCL failures are LHPC_RCCL_STATUS_BASE + ncclResult_t.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <random>
#include <cstring>
#include <new>
#include <vector>

#include "lhpc_common.hpp"
#include "lhpc_rccl.hpp"
#include "lhpc_spmv_impl.hpp"

#define LHPC_NCCL_TRY(expr)                                                \
  do {                                                                     \
    ncclResult_t _r = (expr);                                              \
    if (_r != ncclSuccess) return LHPC_RCCL_STATUS_BASE + static_cast<int>(_r); \
  } while (0)

static_assert(sizeof(ncclUniqueId) == LHPC_DIST_UNIQUE_ID_BYTES, "ncclUniqueId is 128 bytes");

// a registered peer-exchange window: one y buffer, mapped on every rank
struct P2pWindow {
  void *buf = nullptr;              // this rank's y (caller-owned)
  size_t bytes = 0;
  bool ready = false;               // imported: every peer's copy is mapped
  std::vector<void *> peer_base;    // hipIpcOpenMemHandle results (closed on reset)
  void **d_peer_buf = nullptr;      // [nranks] device table of peer pointers (self: own)
  std::vector<void *> peer_buf;     // the same pointers on the host
  std::vector<int64_t> peer_bytes;  // every rank's window size (stencil slabs may differ)
  int64_t min_bytes = 0;            // the smallest of them
  uint64_t narrow = 0;              // bit p: peer p's y has another 16-B phase → 4-B stores
};

struct lhpc_dist_comm {
  ncclComm_t comm = nullptr;  // null for a local (P2P-only) communicator
  int nranks = 1, rank = 0, device = 0;
  hipStream_t s_comm = nullptr;
  // P2P: flags [READY(nranks) | DONE(nranks)] (owned, uncached device
  // memory) shared by every window, the peers' mapped flag arrays, and the
  // windows in export order
  uint32_t *flags = nullptr;
  uint64_t flags_gen = 0;              // identifies this flag allocation (in every blob)
  std::vector<void *> peer_flags_base;
  std::vector<uint64_t> peer_flags_gen;  // the generation of each peer's mapped flags
  uint32_t **d_peer_flags = nullptr;
  bool flags_mapped = false;
  uint32_t *h_status = nullptr;  // host-mapped: bit 0 = a flag wait timed out
  uint32_t epoch = 0;
  uint32_t red_epoch = 0;        // P2P all-gathers of scalars (RED flags)
  int cus = 256;  // compute units of the device
  P2pWindow win[LHPC_DIST_P2P_MAX_WINDOWS];
  int n_win = 0;
  // halo stencil: "u complete on the caller's stream" and "halo planes
  // landed", created on first use and re-recorded by every step
  hipEvent_t ev_in = nullptr, ev_halo = nullptr;
};

struct lhpc_dist_spmv_plan {
  lhpc_dist_comm *comm = nullptr;
  int dtype = LHPC_F32, K = 1;
  int64_t n_rows = 0, n_cols = 0;
  lhpc_options opt{};                       // resolved: the dist_* fields pick the exchange
  std::vector<int64_t> cuts;                // nranks·K + 1 global row cuts
  lhpc::LocalPlans lp;                      // the rank's K blocks (lhpc_multi.hip)
  // the exchange schedules (lhpc_dist_exchange_schedule), entries of chunk k
  // at [first[k], first[k+1])
  std::vector<lhpc_dist_xfer> sched_rccl, sched_p2p;
  std::vector<int64_t> first_rccl, first_p2p;
  // the RCCL calls of sched_rccl, one per entry (lhpc_rccl.hpp; the records
  // lhpc_dist_rccl_calls exports to the CPU tests)
  std::vector<lhpc_rccl_call> calls_rccl;
  std::vector<hipEvent_t> ev;               // [K] chunk k reduced
  std::vector<hipEvent_t> ev_x;             // [K] chunk k's exchange landed (comm stream)
  hipEvent_t done = nullptr;                // last exchange issued on the comm stream
  hipEvent_t ev_p2p = nullptr;              // P2P: READY signalled on the compute stream
  // cross-step overlap (lhpc_dist_spmv_begin): the y of a begun call whose
  // exchange has not been waited for, and whether the local plan can gather
  // x by column parts (part j = the columns exchange j delivers)
  const void *pending_y = nullptr;
  bool chain = false;
  // a pending P2P exchange: its epoch (the peers' DONE values are
  // epoch·64 + chunk + 1), waited for on the compute stream by the consumer
  // (the chained stage per part, or wait_pending for the whole y)
  bool pending_p2p = false;
  uint32_t pending_epoch = 0;
  // chunk reduces alternate over the caller's stream and s_red2
  // (options.dist_reduce_streams), joined by ev_fork / ev_join
  hipStream_t s_red2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  double *h_scalars = nullptr;  // lhpc_dist_cg_solve: 2 pinned host scalars (first solve; freed with the plan)
};

namespace {

ncclDataType_t nccl_dt(int dtype) { return dtype == LHPC_F64 ? ncclFloat64 : ncclFloat32; }

// the schedule of every chunk (see include/lhpc.h lhpc_dist_exchange_schedule)
int build_schedule(const int64_t *cuts, int nranks, int K, int rank, int exchange, int broadcast,
                   std::vector<lhpc_dist_xfer> &out, std::vector<int64_t> &first) {
  out.clear();
  first.assign(static_cast<size_t>(K) + 1, 0);
  for (int k = 0; k < K; ++k) {
    first[k] = static_cast<int64_t>(out.size());
    const int64_t b0 = static_cast<int64_t>(k) * nranks;
    if (exchange == LHPC_DIST_EXCHANGE_P2P) {
      const int64_t b = b0 + rank, cnt = cuts[b + 1] - cuts[b];
      if (cnt > 0) out.push_back(lhpc_dist_xfer{k, LHPC_XFER_PUSH, rank, 0, cuts[b], cnt, cuts[b]});
      continue;
    }
    const int64_t cnt0 = cuts[b0 + 1] - cuts[b0];
    bool equal = !broadcast;
    for (int r = 1; r < nranks && equal; ++r) equal = cuts[b0 + r + 1] - cuts[b0 + r] == cnt0;
    if (equal) {
      // uniform rows: the nnz-balanced cuts are equal-row cuts (C2/C3)
      if (cnt0 > 0) out.push_back(lhpc_dist_xfer{k, LHPC_XFER_ALLGATHER, -1, 0, cuts[b0], cnt0, cuts[b0 + rank]});
      continue;
    }
    for (int r = 0; r < nranks; ++r) {  // exact slices, no padding
      const int64_t cnt = cuts[b0 + r + 1] - cuts[b0 + r];
      if (cnt > 0) out.push_back(lhpc_dist_xfer{k, LHPC_XFER_BROADCAST, r, 1, cuts[b0 + r], cnt, cuts[b0 + r]});
    }
  }
  first[K] = static_cast<int64_t>(out.size());
  return LHPC_OK;
}

// The flag allocation (uncached, one IPC handle): READY [0, n) | DONE
// [n, 2n) | RED [2n, 3n) uint32 flags (n ≤ 64) in the first kFlagBytes, then
// the scalar slots of the P2P all-gather: double [2 parities][64 ranks][8]
constexpr size_t kFlagBytes = 1024;
// uint32 index in the flag allocation of the push kernels' block counters
// (this rank's only; past READY | DONE | RED at ≤ 3·64): y pushes at
// kPushCtr, the stencil's two halo transfers at kPushCtr + 1 and + 2
constexpr int kPushCtr = 192;
static_assert((kPushCtr + 2) * 4 < static_cast<int>(kFlagBytes), "push counters inside the flag words");

// ---- P2P window kernels.  Every kernel of a call reads the status word
// first: once a wait has timed out, pushes and DONE flags are skipped (the
// peers then time out as well), so no rank writes into a peer that never
// declared its y free, and no call reports a half-exchanged y as done.
__device__ __forceinline__ bool p2p_failed(const uint32_t *status) {
  return __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}
// flag store into every peer's flag array at `slot` (READY: rank, DONE:
// nranks + rank), release at system scope: everything this stream did
// before is visible to the peer first
__global__ void k_p2p_signal(uint32_t *const *peer_flags, int slot, uint32_t e, int nranks, int self,
                             const uint32_t *status) {
  const int p = threadIdx.x;
  if (p2p_failed(status)) return;
  if (p < nranks && p != self) __hip_atomic_store(peer_flags[p] + slot, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// wait until every peer's flag at base + p reached epoch e; bounded (~8 s):
// a missing peer sets status bit 0 instead of hanging the device
__global__ void k_p2p_wait(const uint32_t *flags, int base, uint32_t e, int nranks, int self, uint32_t *status) {
  const int p = threadIdx.x;
  if (p >= nranks || p == self) return;
  for (uint32_t spins = 0;; ++spins) {
    const uint32_t f = __hip_atomic_load(flags + base + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (static_cast<int32_t>(f - e) >= 0) return;
    if (spins > (1u << 21) || p2p_failed(status)) {
      __hip_atomic_fetch_or(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(127);
  }
}
// READY to the peers in `mask` only (the stencil's neighbours)
__global__ void k_p2p_signal_mask(uint32_t *const *peer_flags, int slot, uint32_t e, int nranks, int self,
                                  uint64_t mask, const uint32_t *status) {
  const int p = threadIdx.x;
  if (p2p_failed(status)) return;
  if (p < nranks && p != self && ((mask >> p) & 1u))
    __hip_atomic_store(peer_flags[p] + slot, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_p2p_wait_mask(const uint32_t *flags, int base, uint32_t e, int nranks, int self, uint64_t mask,
                                uint32_t *status) {
  const int p = threadIdx.x;
  if (p >= nranks || p == self || !((mask >> p) & 1u)) return;
  for (uint32_t spins = 0;; ++spins) {
    const uint32_t f = __hip_atomic_load(flags + base + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (static_cast<int32_t>(f - e) >= 0) return;
    if (spins > (1u << 21) || p2p_failed(status)) {
      __hip_atomic_fetch_or(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(127);
  }
}

// Halo planes straight into the neighbours' ghost planes: transfer i =
// blockIdx.y (≤ 2: down to rank − 1, up to rank + 1) copies bytes[i] from
// src[i] to dst[i] (a peer's window), 16 B per lane when vec[i], else words;
// then, as k_p2p_push, the transfer's last block signals DONE = v into that
// peer's flag nranks + self (its own block counter kPushCtr + 1 + i)
struct HaloPut {
  const unsigned char *src[2];
  unsigned char *dst[2];
  int64_t bytes[2];
  int peer[2];
  int vec[2];
};
__global__ __launch_bounds__(256) void k_p2p_halo_put(HaloPut h, const uint32_t *status, uint32_t *flags,
                                                      uint32_t *const *peer_flags, int nranks, int self, uint32_t v) {
  const int i = blockIdx.y;
  if (!p2p_failed(status)) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x,
                  T = static_cast<int64_t>(gridDim.x) * blockDim.x;
    if (h.vec[i]) {
      for (int64_t o = 16 * t; o < h.bytes[i]; o += 16 * T)
        *reinterpret_cast<uint4 *>(h.dst[i] + o) = *reinterpret_cast<const uint4 *>(h.src[i] + o);
    } else {
      for (int64_t o = 4 * t; o < h.bytes[i]; o += 4 * T)
        *reinterpret_cast<uint32_t *>(h.dst[i] + o) = *reinterpret_cast<const uint32_t *>(h.src[i] + o);
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t *ctr = flags + kPushCtr + 1 + i;
    if (__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u == gridDim.x) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      if (!p2p_failed(status))
        __hip_atomic_store(peer_flags[h.peer[i]] + nranks + self, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// the consumer's side of a P2P chunk (compute stream, right before the first
// read of it): every block waits for every peer's DONE at base + p ≥ e
// (bounded as k_p2p_wait), then acquires at system scope.  The peers' stores
// reached this GPU's memory over xGMI without passing its L2s, so a line of
// y that an XCD's L2 still holds from before (the gather reads y as the next
// x) could be stale: kP2pAcqBlocks blocks, dealt round-robin over the XCDs,
// make every XCD drop them.  A handful of spinning waves, not one per CU (a
// wave slot per CU would cost a concurrent reduce a block per CU).
constexpr int kP2pAcqBlocks = 16;
__global__ void k_p2p_wait_acquire(const uint32_t *flags, int base, uint32_t e, int nranks, int self,
                                   uint32_t *status, uint64_t mask) {
  const int p = threadIdx.x;
  if (p < nranks && p != self && ((mask >> p) & 1u)) {
    for (uint32_t spins = 0;; ++spins) {
      const uint32_t f = __hip_atomic_load(flags + base + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (static_cast<int32_t>(f - e) >= 0) break;
      if (spins > (1u << 21) || p2p_failed(status)) {
        __hip_atomic_fetch_or(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(127);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

constexpr int kRedMax = 8;
constexpr size_t kFlagAlloc = kFlagBytes + 2 * 64 * kRedMax * sizeof(double);
__device__ __forceinline__ double *red_slots(uint32_t *flags) {
  return reinterpret_cast<double *>(reinterpret_cast<unsigned char *>(flags) + kFlagBytes);
}
// this rank's `count` values into slot [parity][self] of every rank (itself
// included), then its RED flag (epoch e, release) into every peer
__global__ void k_p2p_red_push(uint32_t *const *peer_flags, int nranks, int self, int parity, const double *vals,
                               int count, uint32_t e, const uint32_t *status) {
  const int p = threadIdx.x;
  if (p >= nranks || p2p_failed(status)) return;
  double *dst = red_slots(peer_flags[p]) + (parity * 64 + self) * kRedMax;
  for (int i = 0; i < count; ++i)
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(dst + i),
                       static_cast<unsigned long long>(__double_as_longlong(vals[i])), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if (p != self)
    __hip_atomic_store(peer_flags[p] + 2 * nranks + self, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  else
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}
// after every peer's RED flag: out[r·count + i] = rank r's value i
__global__ void k_p2p_red_collect(uint32_t *flags, int nranks, int parity, int count, double *out) {
  const int t = threadIdx.x;
  if (t >= nranks * count) return;
  const int r = t / count, i = t % count;
  const double *src = red_slots(flags) + (parity * 64 + r) * kRedMax + i;
  out[t] = __longlong_as_double(static_cast<long long>(__hip_atomic_load(
      reinterpret_cast<const unsigned long long *>(src), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)));
}
// out[i] = Σ_r gathered[r·count + i] in rank order (identical on every rank)
__global__ void k_sum_ranks(const double *gathered, int nranks, int count, double *out) {
  const int i = threadIdx.x;
  if (i >= count) return;
  double acc = 0.0;
  for (int r = 0; r < nranks; ++r) acc += gathered[r * count + i];
  out[i] = acc;
}
// bytes [o0, o1) of this rank's y into the same bytes of every peer's y;
// offsets are multiples of 4.  16-B stores on [a0, a1) (the 16-B aligned
// interior) for peers whose y has our 16-B phase, head [o0, a0) and tail
// [a1, o1) as words; a peer with another phase (bit p of `narrow`) gets
// words throughout.  blockIdx.y = peer
// The chunk's DONE signal rides on the push: every block fences its stores at
// system scope and counts itself in (kPushCtr, acq_rel); the last block resets
// the counter and stores DONE = v (release, system scope) into every peer's
// flag nranks + self.  A failed exchange still counts, so the counter stays
// consistent, but stores nothing and signals nothing.
__global__ __launch_bounds__(256) void k_p2p_push(void *const *peer_buf, const unsigned char *y, int64_t o0,
                                                  int64_t o1, int self, uint64_t narrow, const uint32_t *status,
                                                  uint32_t *flags, uint32_t *const *peer_flags, int nranks,
                                                  uint32_t v) {
  if (!p2p_failed(status)) {
    const int p = static_cast<int>(blockIdx.y) + (static_cast<int>(blockIdx.y) >= self ? 1 : 0);
    unsigned char *dst = static_cast<unsigned char *>(peer_buf[p]);
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x,
                  T = static_cast<int64_t>(gridDim.x) * blockDim.x;
    const uintptr_t yb = reinterpret_cast<uintptr_t>(y);
    int64_t a0 = static_cast<int64_t>(((yb + o0 + 15) & ~uintptr_t{15}) - yb);
    int64_t a1 = static_cast<int64_t>(((yb + o1) & ~uintptr_t{15}) - yb);
    if ((narrow >> p) & 1u || a0 >= a1) a0 = a1 = o1;  // words only
    for (int64_t i = o0 + 4 * t; i < a0; i += 4 * T)  // head words
      *reinterpret_cast<uint32_t *>(dst + i) = *reinterpret_cast<const uint32_t *>(y + i);
    for (int64_t i = a0 + 16 * t; i < a1; i += 16 * T)
      *reinterpret_cast<uint4 *>(dst + i) = *reinterpret_cast<const uint4 *>(y + i);
    for (int64_t i = a1 + 4 * t; i < o1; i += 4 * T)  // tail words
      *reinterpret_cast<uint32_t *>(dst + i) = *reinterpret_cast<const uint32_t *>(y + i);
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t *ctr = flags + kPushCtr;
    const uint32_t total = gridDim.x * gridDim.y;
    if (__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u == total) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      if (!p2p_failed(status))
        for (int q = 0; q < nranks; ++q)
          if (q != self)
            __hip_atomic_store(peer_flags[q] + nranks + self, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

struct P2pBlob {  // LHPC_DIST_P2P_BLOB_BYTES per rank
  hipIpcMemHandle_t buf, flags;
  int64_t offset;  // y − its allocation's base
  int64_t bytes;
  uint64_t magic;
  int32_t window;  // export order
  int32_t nranks;
  uint64_t flags_gen;  // changes when the exporter re-allocates its flags (after a reset)
};
static_assert(sizeof(P2pBlob) <= LHPC_DIST_P2P_BLOB_BYTES, "blob size");
constexpr uint64_t kP2pMagic = 0x6c687063705033ull;  // "lhpcP3"

void window_release(P2pWindow &w) {
  for (void *b : w.peer_base)
    if (b) (void)hipIpcCloseMemHandle(b);
  w.peer_base.clear();
  if (w.d_peer_buf) (void)hipFree(w.d_peer_buf);
  w = P2pWindow{};
}

void p2p_release(lhpc_dist_comm *c) {
  for (int i = 0; i < c->n_win; ++i) window_release(c->win[i]);
  c->n_win = 0;
  for (void *b : c->peer_flags_base)
    if (b) (void)hipIpcCloseMemHandle(b);
  c->peer_flags_base.clear();
  c->peer_flags_gen.clear();
  if (c->d_peer_flags) (void)hipFree(c->d_peer_flags);
  if (c->flags) (void)hipFree(c->flags);
  if (c->h_status) (void)hipHostFree(c->h_status);
  c->d_peer_flags = nullptr;
  c->flags = nullptr;
  c->h_status = nullptr;
  c->flags_mapped = false;
  c->epoch = 0;
}

// the ready window whose buffer is y, or null
const P2pWindow *find_window(const lhpc_dist_comm *c, const void *y, size_t need) {
  for (int i = 0; i < c->n_win; ++i)
    if (c->win[i].ready && c->win[i].buf == y && c->win[i].min_bytes >= static_cast<int64_t>(need)) return &c->win[i];
  return nullptr;
}

// the P2P exchange of one call (see the header comment); s = compute stream.
// The host check of the status word sees the timeouts of calls that have
// completed (the caller synchronised); a timeout still in flight is caught on
// the device (the kernels skip) and by the next synchronised check.
int p2p_exchange_begin(lhpc_dist_comm *c, hipStream_t s, hipEvent_t ev) {
  if (*c->h_status) return LHPC_ERR_INTERNAL;  // an earlier flag wait timed out
  ++c->epoch;
  if (c->epoch == 0) c->epoch = 1;
  hipLaunchKernelGGL(k_p2p_signal, dim3(1), dim3(64), 0, s, c->d_peer_flags, c->rank, c->epoch, c->nranks, c->rank,
                     c->h_status);
  LHPC_HIP_TRY(hipGetLastError());
  LHPC_HIP_TRY(hipEventRecord(ev, s));
  LHPC_HIP_TRY(hipStreamWaitEvent(c->s_comm, ev, 0));
  hipLaunchKernelGGL(k_p2p_wait, dim3(1), dim3(64), 0, c->s_comm, c->flags, 0, c->epoch, c->nranks, c->rank,
                     c->h_status);
  return static_cast<int>(hipGetLastError());
}

// chunk j's DONE value: epoch·64 + j + 1, so one slot per rank carries the
// chunk progress of the call
uint32_t p2p_done_value(const lhpc_dist_comm *c, int j) { return c->epoch * 64u + static_cast<uint32_t>(j) + 1u; }

// bytes [o0, o1) of this rank's y to every peer, then DONE(j) (fused, see
// k_p2p_push); a P2P chunk has at most one push (its own block)
int p2p_push(lhpc_dist_comm *c, const P2pWindow *w, int64_t o0, int64_t o1, int j) {
  const int64_t vec = (o1 - o0) / 16 + 1;
  const unsigned bx = static_cast<unsigned>(std::min<int64_t>(64, (vec + 255) / 256));
  hipLaunchKernelGGL(k_p2p_push, dim3(bx, static_cast<unsigned>(c->nranks - 1)), dim3(256), 0, c->s_comm,
                     w->d_peer_buf, static_cast<const unsigned char *>(w->buf), o0, o1, c->rank, w->narrow,
                     c->h_status, c->flags, c->d_peer_flags, c->nranks, p2p_done_value(c, j));
  return static_cast<int>(hipGetLastError());
}

// chunk j with no rows on this rank: DONE(j) alone (a push signals it)
int p2p_signal_done(lhpc_dist_comm *c, int j) {
  hipLaunchKernelGGL(k_p2p_signal, dim3(1), dim3(64), 0, c->s_comm, c->d_peer_flags, c->nranks + c->rank,
                     p2p_done_value(c, j), c->nranks, c->rank, c->h_status);
  return static_cast<int>(hipGetLastError());
}

// on the consumer's stream: every peer's chunk j of the exchange of `epoch`
// has landed, and this GPU's caches hold no stale line of it
int p2p_wait_chunk(lhpc_dist_comm *c, uint32_t epoch, int j, hipStream_t s) {
  const uint32_t v = epoch * 64u + static_cast<uint32_t>(j) + 1u;
  hipLaunchKernelGGL(k_p2p_wait_acquire, dim3(kP2pAcqBlocks), dim3(64), 0, s, c->flags, c->nranks, v, c->nranks,
                     c->rank, c->h_status, ~uint64_t{0});
  return static_cast<int>(hipGetLastError());
}

void destroy_spmv(lhpc_dist_spmv_plan *d) {
  if (!d) return;
  (void)hipSetDevice(d->comm ? d->comm->device : 0);
  lhpc::local_plans_destroy(d->lp);
  for (hipEvent_t e : d->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : d->ev_x)
    if (e) (void)hipEventDestroy(e);
  if (d->done) (void)hipEventDestroy(d->done);
  if (d->ev_fork) (void)hipEventDestroy(d->ev_fork);
  if (d->ev_join) (void)hipEventDestroy(d->ev_join);
  if (d->s_red2) {
    (void)hipStreamSynchronize(d->s_red2);
    (void)hipStreamDestroy(d->s_red2);
  }
  if (d->h_scalars) (void)hipHostFree(d->h_scalars);
  if (d->ev_p2p) (void)hipEventDestroy(d->ev_p2p);
  delete d;
}

// chunk k's RCCL transfers from the schedule: one in-place all-gather, or
// one group of in-place broadcasts (root r sends its block) — the records of
// lhpc_rccl.hpp, with their group brackets
int issue_rccl_chunk(const lhpc_dist_spmv_plan *d, int k, void *y, hipStream_t cs) {
  return lhpc::rccl_issue_list(d->calls_rccl.data(), d->first_rccl[k], d->first_rccl[k + 1], static_cast<unsigned char *>(y),
                         d->comm->comm, cs);
}

// which exchange a call with this y runs (LHPC_DIST_EXCHANGE_NONE: none);
// *win = the peer window for P2P
int pick_exchange(const lhpc_dist_spmv_plan *d, const void *y, const P2pWindow **win) {
  const lhpc_dist_comm *c = d->comm;
  const size_t tsz = d->dtype == LHPC_F64 ? 8 : 4;
  const P2pWindow *w = c->nranks > 1 ? find_window(c, y, static_cast<size_t>(d->n_rows) * tsz) : nullptr;
  *win = nullptr;
  int x = d->opt.dist_exchange;
  if (x == LHPC_DIST_EXCHANGE_NONE) return x;
  if (c->nranks == 1) return d->opt.dist_world1 && c->comm ? LHPC_DIST_EXCHANGE_RCCL : LHPC_DIST_EXCHANGE_NONE;
  if (x == LHPC_DIST_EXCHANGE_AUTO) x = w ? LHPC_DIST_EXCHANGE_P2P : LHPC_DIST_EXCHANGE_RCCL;
  if (x == LHPC_DIST_EXCHANGE_P2P) {
    if (!w) return LHPC_ERR_INVALID_ARG;  // y is not a registered window
    *win = w;
    return x;
  }
  return c->comm ? LHPC_DIST_EXCHANGE_RCCL : LHPC_ERR_INVALID_ARG;  // a local comm has no RCCL
}

// chunk k's exchange on the comm stream, after the compute stream's event;
// ev_x[k] marks this rank's part of it done (RCCL: the chunk landed; P2P: the
// push issued — the peers' chunk is waited for by p2p_wait_chunk)
int exchange_chunk(lhpc_dist_spmv_plan *d, int xk, const P2pWindow *w, int k, void *y, hipStream_t s) {
  lhpc_dist_comm *c = d->comm;
  LHPC_HIP_TRY(hipEventRecord(d->ev[k], s));
  LHPC_HIP_TRY(hipStreamWaitEvent(c->s_comm, d->ev[k], 0));
  lhpc::RocTxRange rb("lhpc_dist_spmv: y chunk exchange");
  if (xk == LHPC_DIST_EXCHANGE_P2P) {
    const int64_t tsz = d->dtype == LHPC_F64 ? 8 : 4;
    // the push signals DONE(k); the consumer waits for the peers' DONE(k) on
    // its own stream (p2p_wait_chunk), so the comm stream carries one kernel
    // per chunk
    bool pushed = false;
    for (int64_t e = d->first_p2p[k]; e < d->first_p2p[k + 1]; ++e) {  // ≤ 1 (build_schedule)
      const lhpc_dist_xfer &x = d->sched_p2p[e];
      if (x.count <= 0 || c->nranks < 2) continue;
      LHPC_TRY(p2p_push(c, w, x.offset * tsz, (x.offset + x.count) * tsz, k));
      pushed = true;
    }
    if (!pushed && c->nranks > 1) LHPC_TRY(p2p_signal_done(c, k));
  } else {
    LHPC_TRY(issue_rccl_chunk(d, k, y, c->s_comm));
  }
  LHPC_HIP_TRY(hipEventRecord(d->ev_x[k], c->s_comm));
  return LHPC_OK;
}

// a begun call's exchange, waited for on `s` (lhpc_dist_spmv_end)
int wait_pending(lhpc_dist_spmv_plan *d, hipStream_t s) {
  if (!d->pending_y) return LHPC_OK;
  d->pending_y = nullptr;
  LHPC_HIP_TRY(hipStreamWaitEvent(s, d->done, 0));  // this rank's own exchange work
  if (d->pending_p2p) {  // the peers' last chunk (DONE values are monotone: all chunks)
    d->pending_p2p = false;
    LHPC_TRY(p2p_wait_chunk(d->comm, d->pending_epoch, d->K - 1, s));
  }
  return LHPC_OK;
}

}  // namespace

extern "C" int lhpc_dist_exchange_schedule(const int64_t *cuts, int nranks, int K, int rank, int exchange,
                                           int broadcast, lhpc_dist_xfer *out, int64_t max_out, int64_t *n_out) {
  try {
    if (!cuts || nranks < 1 || K < 1 || rank < 0 || rank >= nranks || !n_out || max_out < 0 || (max_out > 0 && !out) ||
        (exchange != LHPC_DIST_EXCHANGE_RCCL && exchange != LHPC_DIST_EXCHANGE_P2P))
      return LHPC_ERR_INVALID_ARG;
    const int64_t nb = static_cast<int64_t>(nranks) * K;
    if (cuts[0] != 0) return LHPC_ERR_INVALID_ARG;
    for (int64_t b = 0; b < nb; ++b)
      if (cuts[b + 1] < cuts[b]) return LHPC_ERR_INVALID_ARG;
    std::vector<lhpc_dist_xfer> v;
    std::vector<int64_t> first;
    LHPC_TRY(build_schedule(cuts, nranks, K, rank, exchange, broadcast, v, first));
    *n_out = static_cast<int64_t>(v.size());
    if (static_cast<int64_t>(v.size()) > max_out) return LHPC_ERR_INVALID_ARG;
    if (!v.empty()) std::memcpy(out, v.data(), v.size() * sizeof(lhpc_dist_xfer));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_rccl_calls(const int64_t *cuts, int nranks, int K, int rank, int broadcast, int dtype,
                                    lhpc_rccl_call *out, int64_t max_out, int64_t *n_out) {
  try {
    if (dtype != LHPC_F32 && dtype != LHPC_F64) return LHPC_ERR_INVALID_ARG;
    if (!n_out || max_out < 0 || (max_out > 0 && !out)) return LHPC_ERR_INVALID_ARG;
    int64_t ns = 0;  // the schedule's size (a too-small buffer still reports it)
    const int q = lhpc_dist_exchange_schedule(cuts, nranks, K, rank, LHPC_DIST_EXCHANGE_RCCL, broadcast, nullptr, 0, &ns);
    if (q != LHPC_OK && ns == 0) return q;  // bad cuts / ranks
    std::vector<lhpc_dist_xfer> v(static_cast<size_t>(ns));
    LHPC_TRY(lhpc_dist_exchange_schedule(cuts, nranks, K, rank, LHPC_DIST_EXCHANGE_RCCL, broadcast, v.data(), ns, &ns));
    std::vector<lhpc_rccl_call> calls;
    lhpc::rccl_calls_of(v.data(), ns, dtype, calls);
    *n_out = static_cast<int64_t>(calls.size());
    if (*n_out > max_out) return LHPC_ERR_INVALID_ARG;
    if (!calls.empty()) std::memcpy(out, calls.data(), calls.size() * sizeof(lhpc_rccl_call));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_chain_parts(const int64_t *cuts, int nranks, int K, int64_t n_cols, int64_t tile_width,
                                     int32_t *part, int64_t n_tiles) {
  try {
    if (!cuts || nranks < 1 || K < 1 || n_cols < 0 || tile_width < 1 || !part ||
        n_tiles < (n_cols + tile_width - 1) / tile_width)
      return LHPC_ERR_INVALID_ARG;
    std::vector<int64_t> col_end(static_cast<size_t>(K));
    for (int j = 0; j < K; ++j) col_end[static_cast<size_t>(j)] = cuts[static_cast<int64_t>(j + 1) * nranks];
    for (int j = 0; j < K; ++j)
      if (j > 0 && col_end[j] < col_end[j - 1]) return LHPC_ERR_INVALID_ARG;
    if (col_end[K - 1] < n_cols) return LHPC_ERR_INVALID_ARG;  // the chunks must cover x
    for (int64_t t = 0; t < n_tiles; ++t)
      part[t] = static_cast<int32_t>(lhpc::xtile_part_of_tile(t, tile_width, n_cols, col_end.data(), K));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_get_unique_id(unsigned char *id_out) {
  try {
    if (!id_out) return LHPC_ERR_INVALID_ARG;
    ncclUniqueId id;
    LHPC_NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_comm_create(lhpc_dist_comm **out, const unsigned char *id, int nranks, int rank,
                                     int device) {
  try {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks || device < 0) return LHPC_ERR_INVALID_ARG;
    *out = nullptr;
    LHPC_HIP_TRY(hipSetDevice(device));
    auto *c = new (std::nothrow) lhpc_dist_comm();
    if (!c) return LHPC_ERR_ALLOC;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    (void)hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (c->cus < 8) c->cus = 256;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const ncclResult_t st = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (st != ncclSuccess) {
      delete c;
      return LHPC_RCCL_STATUS_BASE + static_cast<int>(st);
    }
    const hipError_t he = hipStreamCreateWithFlags(&c->s_comm, hipStreamNonBlocking);
    if (he != hipSuccess) {
      (void)ncclCommDestroy(c->comm);
      delete c;
      return static_cast<int>(he);
    }
    *out = c;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_comm_create_local(lhpc_dist_comm **out, int nranks, int rank, int device) {
  try {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || device < 0 || nranks > 64) return LHPC_ERR_INVALID_ARG;
    *out = nullptr;
    LHPC_HIP_TRY(hipSetDevice(device));
    auto *c = new (std::nothrow) lhpc_dist_comm();
    if (!c) return LHPC_ERR_ALLOC;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    (void)hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (c->cus < 8) c->cus = 256;
    const hipError_t he = hipStreamCreateWithFlags(&c->s_comm, hipStreamNonBlocking);
    if (he != hipSuccess) {
      delete c;
      return static_cast<int>(he);
    }
    *out = c;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_p2p_export(lhpc_dist_comm *c, void *y, int64_t bytes, unsigned char *blob_out) {
  try {
    if (!c || !y || bytes <= 0 || bytes % 4 || !blob_out || c->nranks > 64) return LHPC_ERR_INVALID_ARG;
    if (c->n_win >= LHPC_DIST_P2P_MAX_WINDOWS) return LHPC_ERR_UNSUPPORTED;
    for (int i = 0; i < c->n_win; ++i)
      if (c->win[i].buf == y) return LHPC_ERR_INVALID_ARG;  // already a window
    lhpc::RocTxRange rx("lhpc_dist_p2p_export");
    LHPC_HIP_TRY(hipSetDevice(c->device));
    P2pBlob b{};
    void *base = nullptr;
    size_t size = 0;
    LHPC_HIP_TRY(hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t *>(&base), &size, y));
    if (static_cast<unsigned char *>(y) + bytes > static_cast<unsigned char *>(base) + size) return LHPC_ERR_INVALID_ARG;
    LHPC_HIP_TRY(hipIpcGetMemHandle(&b.buf, base));
    if (!c->flags) {
      // flags: uncached, so a peer's store is seen by the next poll; zeroed
      LHPC_HIP_TRY(hipExtMallocWithFlags(reinterpret_cast<void **>(&c->flags), kFlagAlloc, hipDeviceMallocUncached));
      LHPC_HIP_TRY(hipMemset(c->flags, 0, kFlagAlloc));
      c->red_epoch = 0;
      LHPC_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c->h_status), sizeof(uint32_t), hipHostMallocMapped));
      *c->h_status = 0;
      c->epoch = 0;
      static std::atomic<uint64_t> counter{0};
      c->flags_gen = (std::random_device{}() * 0x9E3779B97F4A7C15ull) ^ (++counter << 1) ^ reinterpret_cast<uintptr_t>(c->flags);
      if (c->flags_gen == 0) c->flags_gen = 1;
    }
    LHPC_HIP_TRY(hipIpcGetMemHandle(&b.flags, c->flags));
    b.offset = static_cast<unsigned char *>(y) - static_cast<unsigned char *>(base);
    b.bytes = bytes;
    b.magic = kP2pMagic;
    b.window = c->n_win;
    b.nranks = c->nranks;
    b.flags_gen = c->flags_gen;
    P2pWindow &w = c->win[c->n_win++];
    w = P2pWindow{};
    w.buf = y;
    w.bytes = static_cast<size_t>(bytes);
    std::memset(blob_out, 0, LHPC_DIST_P2P_BLOB_BYTES);
    std::memcpy(blob_out, &b, sizeof(b));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_p2p_import(lhpc_dist_comm *c, const unsigned char *blobs) {
  try {
    if (!c || !blobs || !c->flags) return LHPC_ERR_INVALID_ARG;
    lhpc::RocTxRange rx("lhpc_dist_p2p_import");
    LHPC_HIP_TRY(hipSetDevice(c->device));
    const int nr = c->nranks;
    std::vector<P2pBlob> bl(static_cast<size_t>(nr));
    for (int r = 0; r < nr; ++r) std::memcpy(&bl[r], blobs + static_cast<size_t>(r) * LHPC_DIST_P2P_BLOB_BYTES, sizeof(P2pBlob));
    const int wi = bl[c->rank].window;
    if (wi < 0 || wi >= c->n_win) return LHPC_ERR_INVALID_ARG;
    P2pWindow &w = c->win[wi];
    if (w.ready) return LHPC_ERR_INVALID_ARG;  // imported already
    for (int r = 0; r < nr; ++r)
      if (bl[r].magic != kP2pMagic || bl[r].window != wi || bl[r].nranks != nr || bl[r].bytes <= 0)
        return LHPC_ERR_INVALID_ARG;  // every rank must export the same windows in the same order
    // open everything first; on any failure close what this call opened
    std::vector<void *> pb(static_cast<size_t>(nr), nullptr), pf(static_cast<size_t>(nr), nullptr);
    void **d_buf = nullptr;
    uint32_t **d_flg = nullptr;
    auto undo = [&](int st) {
      for (int r = 0; r < nr; ++r) {
        if (pb[r]) (void)hipIpcCloseMemHandle(pb[r]);
        if (pf[r]) (void)hipIpcCloseMemHandle(pf[r]);
      }
      if (d_buf) (void)hipFree(d_buf);
      if (d_flg) (void)hipFree(d_flg);
      return st;
    };
    std::vector<void *> bufs(static_cast<size_t>(nr), nullptr), flg(static_cast<size_t>(nr), nullptr);
    uint64_t narrow = 0;
    const uintptr_t my_phase = reinterpret_cast<uintptr_t>(w.buf) & 15;
    // the peers' flag arrays: mapped by the first import, and again whenever a
    // peer's blob carries another flags generation (it reset and re-exported)
    bool remap = !c->flags_mapped;
    for (int r = 0; r < nr && !remap; ++r)
      if (r != c->rank && c->peer_flags_gen[static_cast<size_t>(r)] != bl[r].flags_gen) remap = true;
    for (int r = 0; r < nr; ++r) {
      if (r == c->rank) {
        bufs[r] = w.buf;
        flg[r] = c->flags;
        continue;
      }
      hipError_t e = hipIpcOpenMemHandle(&pb[r], bl[r].buf, hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) return undo(static_cast<int>(e));
      bufs[r] = static_cast<unsigned char *>(pb[r]) + bl[r].offset;
      if ((reinterpret_cast<uintptr_t>(bufs[r]) & 15) != my_phase) narrow |= uint64_t{1} << r;
      if (remap) {
        if (c->flags_mapped && c->peer_flags_gen[static_cast<size_t>(r)] == bl[r].flags_gen) {
          flg[r] = c->peer_flags_base[static_cast<size_t>(r)];  // unchanged: keep the mapping
          continue;
        }
        e = hipIpcOpenMemHandle(&pf[r], bl[r].flags, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return undo(static_cast<int>(e));
        flg[r] = pf[r];
      }
    }
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&d_buf), nr * sizeof(void *));
    if (e == hipSuccess) e = hipMemcpy(d_buf, bufs.data(), nr * sizeof(void *), hipMemcpyHostToDevice);
    if (e == hipSuccess && remap) {
      e = hipMalloc(reinterpret_cast<void **>(&d_flg), nr * sizeof(void *));
      if (e == hipSuccess) e = hipMemcpy(d_flg, flg.data(), nr * sizeof(void *), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) return undo(static_cast<int>(e));
    // commit
    w.peer_base = pb;
    w.d_peer_buf = d_buf;
    w.peer_buf = bufs;
    w.peer_bytes.assign(static_cast<size_t>(nr), 0);
    w.min_bytes = INT64_MAX;
    for (int r = 0; r < nr; ++r) {
      w.peer_bytes[static_cast<size_t>(r)] = bl[r].bytes;
      w.min_bytes = std::min<int64_t>(w.min_bytes, bl[r].bytes);
    }
    w.narrow = narrow;
    w.ready = true;
    if (remap) {
      // close the replaced peer mappings (every window's kernels read peers'
      // flags through d_peer_flags only, which is swapped here).  Kernels on the
      // callers' compute streams (k_p2p_signal, k_p2p_signal_mask,
      // k_p2p_red_push) dereference the old table too, and their streams are not
      // known here: drain the whole device before the old mappings close
      // (import is a setup call, not on the step path)
      if (c->flags_mapped) (void)hipDeviceSynchronize();
      else if (c->s_comm) (void)hipStreamSynchronize(c->s_comm);
      std::vector<void *> base(static_cast<size_t>(nr), nullptr);
      for (int r = 0; r < nr; ++r) {
        if (r == c->rank) continue;
        void *old = c->flags_mapped ? c->peer_flags_base[static_cast<size_t>(r)] : nullptr;
        if (pf[r]) {
          if (old) (void)hipIpcCloseMemHandle(old);
          base[static_cast<size_t>(r)] = pf[r];
        } else {
          base[static_cast<size_t>(r)] = old;
        }
      }
      if (c->d_peer_flags) (void)hipFree(c->d_peer_flags);
      c->peer_flags_base = base;
      c->peer_flags_gen.assign(static_cast<size_t>(nr), 0);
      for (int r = 0; r < nr; ++r) c->peer_flags_gen[static_cast<size_t>(r)] = bl[r].flags_gen;
      c->d_peer_flags = d_flg;
      c->flags_mapped = true;
    }
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_p2p_unmap(lhpc_dist_comm *c, void *y) {
  try {
    if (!c || !y || c->n_win == 0 || c->win[c->n_win - 1].buf != y) return LHPC_ERR_INVALID_ARG;
    LHPC_HIP_TRY(hipSetDevice(c->device));
    if (c->s_comm) LHPC_HIP_TRY(hipStreamSynchronize(c->s_comm));
    window_release(c->win[--c->n_win]);
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_p2p_reset(lhpc_dist_comm *c) {
  try {
    if (!c) return LHPC_ERR_INVALID_ARG;
    LHPC_HIP_TRY(hipSetDevice(c->device));
    if (c->s_comm) LHPC_HIP_TRY(hipStreamSynchronize(c->s_comm));
    p2p_release(c);
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_p2p_status(const lhpc_dist_comm *c) {
  try {
    if (!c) return LHPC_ERR_INVALID_ARG;
    return c->h_status && *c->h_status ? LHPC_ERR_INTERNAL : LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_comm_destroy(lhpc_dist_comm *c) {
  try {
    if (!c) return LHPC_OK;
    (void)hipSetDevice(c->device);
    if (c->s_comm) (void)hipStreamSynchronize(c->s_comm);
    p2p_release(c);
    int st = LHPC_OK;
    if (c->comm) {
      const ncclResult_t r = ncclCommDestroy(c->comm);
      if (r != ncclSuccess) st = LHPC_RCCL_STATUS_BASE + static_cast<int>(r);
    }
    if (c->s_comm) (void)hipStreamDestroy(c->s_comm);
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->ev_halo) (void)hipEventDestroy(c->ev_halo);
    delete c;
    return st;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_comm_info(const lhpc_dist_comm *c, int *nranks, int *rank, int *device) {
  try {
    if (!c) return LHPC_ERR_INVALID_ARG;
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    if (device) *device = c->device;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

namespace {
// out[r·count + i] = rank r's vals[i], on `s`: RCCL all-gather, or over a
// P2P communicator the scalar slots of the flag allocation (count ≤ 8;
// double-buffered by parity: a rank overwrites parity p only after every
// peer signalled the reduction after the one that last read it)
int allgather_f64(lhpc_dist_comm *c, const double *vals, int count, double *out, hipStream_t s) {
  if (c->nranks == 1) {
    LHPC_HIP_TRY(hipMemcpyAsync(out, vals, static_cast<size_t>(count) * 8, hipMemcpyDeviceToDevice, s));
    return LHPC_OK;
  }
  if (c->comm) {
    LHPC_NCCL_TRY(ncclAllGather(vals, out, static_cast<size_t>(count), ncclFloat64, c->comm, s));
    return LHPC_OK;
  }
  if (!c->flags_mapped || count > kRedMax) return LHPC_ERR_UNSUPPORTED;  // no window imported yet
  if (*c->h_status) return LHPC_ERR_INTERNAL;
  const uint32_t e = ++c->red_epoch;
  const int parity = static_cast<int>(e & 1u);
  hipLaunchKernelGGL(k_p2p_red_push, dim3(1), dim3(64), 0, s, c->d_peer_flags, c->nranks, c->rank, parity, vals, count,
                     e, c->h_status);
  LHPC_HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_p2p_wait, dim3(1), dim3(64), 0, s, c->flags, 2 * c->nranks, e, c->nranks, c->rank,
                     c->h_status);
  LHPC_HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_p2p_red_collect, dim3(1), dim3(512), 0, s, c->flags, c->nranks, parity, count, out);
  return static_cast<int>(hipGetLastError());
}
}  // namespace

extern "C" int lhpc_dist_allgather_f64(lhpc_dist_comm *c, const double *vals, int64_t count, double *out,
                                       void *stream) {
  try {
    if (!c || count < 0 || (count > 0 && (!vals || !out))) return LHPC_ERR_INVALID_ARG;
    if (count == 0) return LHPC_OK;
    LHPC_HIP_TRY(hipSetDevice(c->device));
    if (!c->comm && c->nranks > 1 && count > kRedMax) return LHPC_ERR_UNSUPPORTED;
    return allgather_f64(c, vals, static_cast<int>(count), out, static_cast<hipStream_t>(stream));
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_allreduce_sum_f64(lhpc_dist_comm *c, double *buf, int64_t count, void *stream) {
  try {
    if (!c || (count > 0 && !buf) || count < 0) return LHPC_ERR_INVALID_ARG;
    if (count == 0) return LHPC_OK;
    LHPC_HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (c->comm) {
      LHPC_NCCL_TRY(ncclAllReduce(buf, buf, static_cast<size_t>(count), ncclFloat64, ncclSum, c->comm, s));
      return LHPC_OK;
    }
    // P2P communicator: gather every rank's values, add them in rank order
    if (c->nranks == 1) return LHPC_OK;
    if (count > kRedMax) return LHPC_ERR_UNSUPPORTED;
    double *g = nullptr;
    LHPC_HIP_TRY(lhpc::scratch_alloc(reinterpret_cast<void **>(&g), static_cast<size_t>(c->nranks * count) * 8, s));
    int st = allgather_f64(c, buf, static_cast<int>(count), g, s);
    if (st == LHPC_OK) {
      hipLaunchKernelGGL(k_sum_ranks, dim3(1), dim3(64), 0, s, g, c->nranks, static_cast<int>(count), buf);
      st = static_cast<int>(hipGetLastError());
    }
    (void)hipFreeAsync(g, s);
    return st;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_spmv_plan_create_opts(lhpc_dist_spmv_plan **out, lhpc_dist_comm *comm, int dtype,
                                               int64_t n_rows, int64_t n_cols, int K, const int64_t *cuts,
                                               const void *row_ptr, int row_ptr_bits, const int32_t *col_idx,
                                               const void *val, unsigned flags, const lhpc_options *opts) {
  try {
    if (!out || !comm || !cuts || !row_ptr || K < 1 || n_rows < 0 || n_cols < 0 ||
        (dtype != LHPC_F32 && dtype != LHPC_F64) || (row_ptr_bits != 32 && row_ptr_bits != 64))
      return LHPC_ERR_INVALID_ARG;
    *out = nullptr;
    const int nr = comm->nranks, rk = comm->rank;
    const int64_t nb = static_cast<int64_t>(nr) * K;
    if (cuts[0] != 0 || cuts[nb] != n_rows) return LHPC_ERR_INVALID_ARG;
    for (int64_t b = 0; b < nb; ++b)
      if (cuts[b + 1] < cuts[b]) return LHPC_ERR_INVALID_ARG;
    const lhpc_options o = lhpc::resolve_options(opts);
    if (o.dist_exchange < LHPC_DIST_EXCHANGE_AUTO || o.dist_exchange > LHPC_DIST_EXCHANGE_NONE) return LHPC_ERR_INVALID_ARG;
    if (K > 63) return LHPC_ERR_INVALID_ARG;  // the P2P DONE flag carries the chunk in 6 bits
    LHPC_HIP_TRY(hipSetDevice(comm->device));
    auto *d = new (std::nothrow) lhpc_dist_spmv_plan();
    if (!d) return LHPC_ERR_ALLOC;
    d->comm = comm;
    d->dtype = dtype;
    d->K = K;
    d->n_rows = n_rows;
    d->n_cols = n_cols;
    d->opt = o;
    d->cuts.assign(cuts, cuts + nb + 1);
    build_schedule(cuts, nr, K, rk, LHPC_DIST_EXCHANGE_RCCL, o.dist_broadcast, d->sched_rccl, d->first_rccl);
    lhpc::rccl_calls_of(d->sched_rccl.data(), static_cast<int64_t>(d->sched_rccl.size()), dtype, d->calls_rccl);
    build_schedule(cuts, nr, K, rk, LHPC_DIST_EXCHANGE_P2P, 0, d->sched_p2p, d->first_p2p);
    // the local CSR: the rank's K blocks stacked in chunk order
    std::vector<int64_t> ls(static_cast<size_t>(K) + 1, 0);
    for (int k = 0; k < K; ++k) {
      const int64_t b = static_cast<int64_t>(k) * nr + rk;
      ls[k + 1] = ls[k] + (cuts[b + 1] - cuts[b]);
    }
    int st = lhpc::local_plans_create(d->lp, dtype, n_cols, K, ls.data(), row_ptr, row_ptr_bits, col_idx, val,
                                      comm->device, flags, o);
    // column parts of the stage for chained calls (square matrices: chunk j's
    // rows of y are columns [cuts[j·N], cuts[(j+1)·N]) of the next x)
    if (st == LHPC_OK && n_rows == n_cols) {
      std::vector<int64_t> col_end(static_cast<size_t>(K));
      for (int j = 0; j < K; ++j) col_end[static_cast<size_t>(j)] = cuts[static_cast<int64_t>(j + 1) * nr];
      d->chain = lhpc::local_plans_column_parts(d->lp, col_end.data(), K);
    }
    if (st == LHPC_OK) {
      d->ev.assign(static_cast<size_t>(K), nullptr);
      d->ev_x.assign(static_cast<size_t>(K), nullptr);
      for (auto &e : d->ev_x)
        if (st == LHPC_OK) st = static_cast<int>(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      for (auto &e : d->ev)
        if (st == LHPC_OK) st = static_cast<int>(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      if (st == LHPC_OK) st = static_cast<int>(hipEventCreateWithFlags(&d->done, hipEventDisableTiming));
      const int nstreams = o.dist_reduce_streams > 0 ? o.dist_reduce_streams : 2;
      if (st == LHPC_OK && nstreams > 1 && K > 1) {
        st = static_cast<int>(hipStreamCreateWithFlags(&d->s_red2, hipStreamNonBlocking));
        if (st == LHPC_OK) st = static_cast<int>(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
        if (st == LHPC_OK) st = static_cast<int>(hipEventCreateWithFlags(&d->ev_join, hipEventDisableTiming));
      }
      if (st == LHPC_OK) st = static_cast<int>(hipEventCreateWithFlags(&d->ev_p2p, hipEventDisableTiming));
    }
    if (st != LHPC_OK) {
      destroy_spmv(d);
      return st;
    }
    *out = d;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_spmv_plan_create(lhpc_dist_spmv_plan **out, lhpc_dist_comm *comm, int dtype,
                                          int64_t n_rows, int64_t n_cols, int K, const int64_t *cuts,
                                          const void *row_ptr, int row_ptr_bits, const int32_t *col_idx,
                                          const void *val, unsigned flags) {
  try {
    return lhpc_dist_spmv_plan_create_opts(out, comm, dtype, n_rows, n_cols, K, cuts, row_ptr, row_ptr_bits, col_idx,
                                           val, flags, nullptr);
  } LHPC_ABI_CATCH
}

namespace {
// lhpc_dist_spmv_begin; local_only: this rank's rows of y only (no exchange,
// the CG solver's q = A·p)
int spmv_begin(lhpc_dist_spmv_plan *d, const void *x, void *y, hipStream_t s, bool local_only) {
  if (!d || (d->n_cols > 0 && !x) || (d->n_rows > 0 && !y) || (x == y && d->n_rows > 0)) return LHPC_ERR_INVALID_ARG;
  lhpc_dist_comm *c = d->comm;
  lhpc::RocTxRange rx("lhpc_dist_spmv");
  LHPC_HIP_TRY(hipSetDevice(c->device));
  const size_t tsz = d->dtype == LHPC_F64 ? 8 : 4;
  // the y exchange: direct peer stores into a registered window, RCCL, or none
  const P2pWindow *win = nullptr;
  const int xk = local_only ? LHPC_DIST_EXCHANGE_NONE : pick_exchange(d, y, &win);
  if (xk < 0) return xk;
  // x is the y of the begun call before (chained): its exchange is still in
  // flight; with column parts, part j of the stage waits only for exchange j
  // of that call and runs while the later chunks travel (cross-step overlap),
  // else the stage waits for the whole exchange.  Any other x: the begun
  // call is finished first.
  const bool chained = d->pending_y && d->pending_y == x;
  if (d->pending_y && !chained) LHPC_TRY(wait_pending(d, s));
  if (xk == LHPC_DIST_EXCHANGE_P2P) LHPC_TRY(p2p_exchange_begin(c, s, d->ev_p2p));
  const bool xchg = xk != LHPC_DIST_EXCHANGE_NONE;
  int gathered = 0;  // ranges of a range-gather plan gathered so far (in order)
  if (chained && d->chain) {
    lhpc::RocTxRange rc("lhpc_dist_spmv: chained stage");
    for (int j = 0; j < d->K; ++j) {
      if (d->pending_p2p) LHPC_TRY(p2p_wait_chunk(c, d->pending_epoch, j, s));  // the peers' chunk j
      else LHPC_HIP_TRY(hipStreamWaitEvent(s, d->ev_x[j], 0));
      LHPC_TRY(lhpc::local_plans_stage_part(d->lp, x, j, s));
    }
    // this rank's own pushes of x end before anything here writes its rows
    if (d->pending_p2p) LHPC_HIP_TRY(hipStreamWaitEvent(s, d->done, 0));
    d->pending_y = nullptr;
    d->pending_p2p = false;
  } else {
    if (chained) LHPC_TRY(wait_pending(d, s));
    LHPC_TRY(lhpc::local_plans_stage(d->lp, x, s));
  }
  // two reduce streams: chunk k on s (even k) or s_red2 (odd k), so the next
  // chunk's workgroups take the CUs a chunk's last round leaves idle; range
  // gathers (a range's first entries come from the range before) stay on one
  const bool two = d->s_red2 && d->K > 1 && !d->lp.range_gather();
  if (two) {
    LHPC_HIP_TRY(hipEventRecord(d->ev_fork, s));
    LHPC_HIP_TRY(hipStreamWaitEvent(d->s_red2, d->ev_fork, 0));
  }
  for (int k = 0; k < d->K; ++k) {
    hipStream_t sk = two && (k & 1) ? d->s_red2 : s;
    const int64_t b = static_cast<int64_t>(k) * c->nranks + c->rank;
    void *yk = static_cast<unsigned char *>(y) + d->cuts[b] * tsz;
    LHPC_TRY(lhpc::local_plans_chunk(d->lp, x, k, yk, gathered, sk));
    if (xchg) LHPC_TRY(exchange_chunk(d, xk, win, k, y, sk));
  }
  if (two) {
    LHPC_HIP_TRY(hipEventRecord(d->ev_join, d->s_red2));
    LHPC_HIP_TRY(hipStreamWaitEvent(s, d->ev_join, 0));
  }
  if (xchg) {
    LHPC_HIP_TRY(hipEventRecord(d->done, c->s_comm));
    d->pending_y = y;
    d->pending_p2p = xk == LHPC_DIST_EXCHANGE_P2P;
    d->pending_epoch = c->epoch;
  }
  return LHPC_OK;
}

// the exchange of y alone (y holds this rank's blocks), left in flight like
// a begun call's, so a chained call's stage can wait per chunk
int exchange_begin(lhpc_dist_spmv_plan *d, void *y, hipStream_t s) {
  lhpc_dist_comm *c = d->comm;
  LHPC_TRY(wait_pending(d, s));
  const P2pWindow *win = nullptr;
  const int xk = pick_exchange(d, y, &win);
  if (xk < 0) return xk;
  if (xk == LHPC_DIST_EXCHANGE_NONE) return LHPC_OK;
  if (xk == LHPC_DIST_EXCHANGE_P2P) LHPC_TRY(p2p_exchange_begin(c, s, d->ev_p2p));
  for (int k = 0; k < d->K; ++k) LHPC_TRY(exchange_chunk(d, xk, win, k, y, s));
  LHPC_HIP_TRY(hipEventRecord(d->done, c->s_comm));
  d->pending_y = y;
  d->pending_p2p = xk == LHPC_DIST_EXCHANGE_P2P;
  d->pending_epoch = c->epoch;
  return LHPC_OK;
}
}  // namespace

extern "C" int lhpc_dist_spmv_begin(lhpc_dist_spmv_plan *d, const void *x, void *y, void *stream) {
  try {
    return spmv_begin(d, x, y, static_cast<hipStream_t>(stream), false);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_spmv_plan_info(const lhpc_dist_spmv_plan *d, lhpc_spmv_plan_info *info, int *chained_stage) {
  try {
    if (!d || !info) return LHPC_ERR_INVALID_ARG;
    const lhpc_spmv_plan *q = d->lp.split;
    for (const lhpc_spmv_plan *b : d->lp.block_plan)
      if (!q && b) q = b;
    if (chained_stage) *chained_stage = d->chain ? 1 : 0;
    if (!q) {  // no local rows
      std::memset(info, 0, sizeof(*info));
      info->dtype = d->dtype;
      info->n_cols = d->n_cols;
      info->device = d->comm->device;
      return LHPC_OK;
    }
    return lhpc_spmv_plan_info_get(q, info);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_spmv_end(lhpc_dist_spmv_plan *d, void *stream) {
  try {
    if (!d) return LHPC_ERR_INVALID_ARG;
    LHPC_HIP_TRY(hipSetDevice(d->comm->device));
    return wait_pending(d, static_cast<hipStream_t>(stream));
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_spmv(lhpc_dist_spmv_plan *d, const void *x, void *y, void *stream) {
  try {
    LHPC_TRY(lhpc_dist_spmv_begin(d, x, y, stream));
    return lhpc_dist_spmv_end(d, stream);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_exchange(lhpc_dist_spmv_plan *d, void *y, void *stream) {
  try {
    if (!d || (d->n_rows > 0 && !y)) return LHPC_ERR_INVALID_ARG;
    lhpc::RocTxRange rx("lhpc_dist_exchange");
    LHPC_HIP_TRY(hipSetDevice(d->comm->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    LHPC_TRY(exchange_begin(d, y, s));
    return wait_pending(d, s);
  } LHPC_ABI_CATCH
}

namespace {
__global__ void k_set_scalars(double *p, double v, int n) {
  if (static_cast<int>(threadIdx.x) < n) p[threadIdx.x] = v;
}
// out = Σ_b part[slot(b)] over the N·K global blocks in block order b = k·N + r
// (gathered as [r][K]): the dot is independent of how the blocks are spread
// over ranks, so an N-rank solve matches a one-rank solve of the same split
__global__ void k_sum_blocks(const double *gathered, int nranks, int K, double *out) {
  if (threadIdx.x != 0) return;
  double acc = 0.0;
  for (int k = 0; k < K; ++k)
    for (int r = 0; r < nranks; ++r) acc += gathered[r * K + k];
  *out = acc;
}
}  // namespace

extern "C" int lhpc_dist_cg_solve(lhpc_dist_spmv_plan *d, const void *b, void *x, void *p_work, double tol,
                                  int max_iter, int check_every, int *iters_out, double *resid_out, void *stream) {
  try {
    if (!d || !b || !x || !p_work || max_iter < 0 || !(tol >= 0.0) || d->n_rows != d->n_cols || b == x ||
        p_work == x || p_work == b)
      return LHPC_ERR_INVALID_ARG;
    lhpc_dist_comm *c = d->comm;
    if (d->K > kRedMax) return LHPC_ERR_UNSUPPORTED;  // K dot partials per rank in one all-gather
    lhpc::RocTxRange rx("lhpc_dist_cg_solve");
    LHPC_HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    LHPC_TRY(wait_pending(d, s));
    const int N = c->nranks, K = d->K, dt = d->dtype;
    const int64_t n = d->n_rows;
    const size_t ts = dt == LHPC_F32 ? 4 : 8;
    if (check_every < 1) check_every = 1;
    auto at = [&](const void *v, int64_t i) { return static_cast<unsigned char *>(const_cast<void *>(v)) + i * ts; };
    // this rank's K blocks of rows
    std::vector<int64_t> r0(static_cast<size_t>(K)), len(static_cast<size_t>(K));
    for (int k = 0; k < K; ++k) {
      const int64_t bi = static_cast<int64_t>(k) * N + c->rank;
      r0[static_cast<size_t>(k)] = d->cuts[bi];
      len[static_cast<size_t>(k)] = d->cuts[bi + 1] - d->cuts[bi];
    }
    // scratch: r and q (full length: the SpMV writes q at global rows), the
    // scalars [rr0, rr1, pq, bb, one] and the dot partials / their all-gather
    void *vec = nullptr;
    double *sc = nullptr;
    LHPC_HIP_TRY(lhpc::scratch_alloc(&vec, static_cast<size_t>(std::max<int64_t>(n, 1)) * ts * 2, s));
    struct Free {
      void *a;
      hipStream_t s;
      ~Free() { (void)hipFreeAsync(a, s); }
    } fv{vec, s};
    const int parts = 8 + K + N * K;
    LHPC_HIP_TRY(lhpc::scratch_alloc(reinterpret_cast<void **>(&sc), static_cast<size_t>(parts) * 8, s));
    Free fs{sc, s};
    void *r = vec, *q = at(vec, n);
    double *rr[2] = {sc, sc + 1}, *pq = sc + 2, *bb = sc + 3, *one = sc + 4, *part = sc + 8, *gath = sc + 8 + K;
    hipLaunchKernelGGL(k_set_scalars, dim3(1), dim3(64), 0, s, one, 1.0, 1);
    LHPC_HIP_TRY(hipGetLastError());
    // global dot from this rank's K block partials: all-gather, block-order sum
    auto global_dot = [&](double *out) -> int {
      LHPC_TRY(allgather_f64(c, part, K, gath, s));
      hipLaunchKernelGGL(k_sum_blocks, dim3(1), dim3(64), 0, s, gath, N, K, out);
      return static_cast<int>(hipGetLastError());
    };
    auto dots = [&](const void *a, const void *bv, double *out) -> int {
      for (int k = 0; k < K; ++k) LHPC_TRY(lhpc_vec_dot(dt, len[k], at(a, r0[k]), at(bv, r0[k]), part + k, s));
      return global_dot(out);
    };
    if (!d->h_scalars)
      LHPC_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&d->h_scalars), 2 * sizeof(double), hipHostMallocDefault));
    double &h_rr = d->h_scalars[0], &h_bb = d->h_scalars[1];
    h_rr = h_bb = 0.0;
    // bb = b·b; q = A·x (x complete on every rank); r = b − q; p = r; rr = r·r
    LHPC_TRY(dots(b, b, bb));
    LHPC_TRY(spmv_begin(d, x, q, s, true));
    for (int k = 0; k < K; ++k) {
      if (!len[k]) {
        LHPC_HIP_TRY(hipMemsetAsync(part + k, 0, 8, s));
        continue;
      }
      LHPC_HIP_TRY(hipMemcpyAsync(at(r, r0[k]), at(b, r0[k]), len[k] * ts, hipMemcpyDeviceToDevice, s));
      LHPC_TRY(lhpc_cg_step_r(dt, len[k], one, one, at(r, r0[k]), at(q, r0[k]), part + k, s));
      LHPC_HIP_TRY(hipMemcpyAsync(at(p_work, r0[k]), at(r, r0[k]), len[k] * ts, hipMemcpyDeviceToDevice, s));
    }
    LHPC_TRY(global_dot(rr[0]));
    LHPC_TRY(exchange_begin(d, p_work, s));  // p complete on every rank; the next stage waits per chunk
    LHPC_HIP_TRY(hipMemcpyAsync(&h_bb, bb, 8, hipMemcpyDeviceToHost, s));  // pinned
    LHPC_HIP_TRY(hipMemcpyAsync(&h_rr, rr[0], 8, hipMemcpyDeviceToHost, s));
    LHPC_HIP_TRY(hipStreamSynchronize(s));
    const double stop = tol * tol * (h_bb > 0.0 ? h_bb : 1.0);
    int it = 0, cur = 0, status = LHPC_OK;
    if (h_rr > stop) {
      for (it = 1; it <= max_iter; ++it) {
        // q = A·p: a chained stage (part j of p waits only for exchange j)
        LHPC_TRY(spmv_begin(d, p_work, q, s, true));
        LHPC_TRY(dots(p_work, q, pq));
        for (int k = 0; k < K; ++k) {  // r −= α·q, partial r·r
          if (len[k]) LHPC_TRY(lhpc_cg_step_r(dt, len[k], rr[cur], pq, at(r, r0[k]), at(q, r0[k]), part + k, s));
          else LHPC_HIP_TRY(hipMemsetAsync(part + k, 0, 8, s));
        }
        LHPC_TRY(global_dot(rr[cur ^ 1]));
        if (it % check_every == 0 || it == max_iter) {
          LHPC_HIP_TRY(hipMemcpyAsync(&h_rr, rr[cur ^ 1], 8, hipMemcpyDeviceToHost, s));
          LHPC_HIP_TRY(hipStreamSynchronize(s));
          if (!std::isfinite(h_rr)) {
            status = LHPC_ERR_INTERNAL;  // breakdown: the matrix is not SPD?
            break;
          }
          if (h_rr <= stop) {
            for (int k = 0; k < K; ++k)  // x += α·p
              if (len[k])
                LHPC_TRY(lhpc_cg_step_xp(dt, len[k], rr[cur], pq, nullptr, nullptr, at(x, r0[k]), at(p_work, r0[k]),
                                         nullptr, s));
            break;
          }
        }
        for (int k = 0; k < K; ++k)  // x += α·p; p = r + β·p
          if (len[k])
            LHPC_TRY(lhpc_cg_step_xp(dt, len[k], rr[cur], pq, rr[cur ^ 1], rr[cur], at(x, r0[k]), at(p_work, r0[k]),
                                     at(r, r0[k]), s));
        LHPC_TRY(exchange_begin(d, p_work, s));
        cur ^= 1;
      }
      if (it > max_iter) it = max_iter;
    }
    // every rank ends with the whole x: this rank's rows of x go out through
    // p_work (the registered window when the exchange is P2P)
    LHPC_TRY(wait_pending(d, s));
    for (int k = 0; k < K; ++k)
      if (len[k]) LHPC_HIP_TRY(hipMemcpyAsync(at(p_work, r0[k]), at(x, r0[k]), len[k] * ts, hipMemcpyDeviceToDevice, s));
    LHPC_TRY(exchange_begin(d, p_work, s));
    LHPC_TRY(wait_pending(d, s));
    LHPC_HIP_TRY(hipMemcpyAsync(x, p_work, static_cast<size_t>(n) * ts, hipMemcpyDeviceToDevice, s));
    LHPC_HIP_TRY(hipStreamSynchronize(s));
    if (c->h_status && *c->h_status) status = LHPC_ERR_INTERNAL;  // a P2P flag wait timed out
    if (iters_out) *iters_out = it;
    if (resid_out) *resid_out = std::sqrt(std::max(h_rr, 0.0)) / std::sqrt(h_bb > 0.0 ? h_bb : 1.0);
    return status;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_spmv_plan_destroy(lhpc_dist_spmv_plan *d) {
  try {
    destroy_spmv(d);
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_stencil7_f32_x(lhpc_dist_comm *c, float *u, float *out, int64_t nzl, int64_t ny,
                                        int64_t nx, int64_t ghost, float c0, float c1, int exchange, void *stream) {
  try {
    if (!c || !u || !out || nzl < 1 || ny < 0 || nx < 0 || ghost < 1) return LHPC_ERR_INVALID_ARG;
    if (exchange != LHPC_DIST_EXCHANGE_AUTO && exchange != LHPC_DIST_EXCHANGE_RCCL && exchange != LHPC_DIST_EXCHANGE_P2P)
      return LHPC_ERR_INVALID_ARG;
    LHPC_HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t P = (ny + 2 * ghost) * (nx + 2 * ghost);  // padded plane
    auto plane = [&](int64_t z) { return u + (z + ghost) * P; };  // logical plane z ∈ [−ghost, nzl + ghost)
    const bool lo = c->rank > 0, hi = c->rank < c->nranks - 1;
    lhpc::RocTxRange rx("lhpc_dist_stencil7_f32");
    const bool halo = lo || hi;
    // the exchange: P2P when u is a registered window (AUTO) or asked for
    const size_t ubytes = static_cast<size_t>(nzl + 2 * ghost) * static_cast<size_t>(P) * 4;
    const P2pWindow *w = nullptr;
    if (halo && exchange != LHPC_DIST_EXCHANGE_RCCL) {
      for (int i = 0; i < c->n_win && !w; ++i)
        if (c->win[i].ready && c->win[i].buf == u && c->win[i].bytes >= ubytes) w = &c->win[i];
      if (!w && exchange == LHPC_DIST_EXCHANGE_P2P) return LHPC_ERR_INVALID_ARG;  // u is not a window
    }
    if (halo && !w && !c->comm) return LHPC_ERR_UNSUPPORTED;  // a local communicator has no RCCL
    if (halo) {
      if (!c->ev_in) LHPC_HIP_TRY(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
      if (!c->ev_halo) LHPC_HIP_TRY(hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming));
    }
    uint64_t mask = 0;
    if (w) {
      // READY (epoch) to the neighbours on the compute stream: this rank has
      // finished every earlier read of u's ghost planes
      lhpc::RocTxRange rh("lhpc_dist_stencil7_f32: P2P halo");
      if (*c->h_status) return LHPC_ERR_INTERNAL;  // an earlier flag wait timed out
      const int64_t pb = P * 4;
      int64_t nzl_lo = 0;  // the lower neighbour's slab depth, from its window size
      if (lo) {
        const int64_t wb = w->peer_bytes[static_cast<size_t>(c->rank - 1)];
        if (wb % pb || wb / pb - 2 * ghost < 1) return LHPC_ERR_INVALID_ARG;
        nzl_lo = wb / pb - 2 * ghost;
      }
      if (hi && w->peer_bytes[static_cast<size_t>(c->rank + 1)] < (2 * ghost + 1) * pb) return LHPC_ERR_INVALID_ARG;
      if (lo) mask |= uint64_t{1} << (c->rank - 1);
      if (hi) mask |= uint64_t{1} << (c->rank + 1);
      ++c->epoch;
      if (c->epoch == 0) c->epoch = 1;
      hipLaunchKernelGGL(k_p2p_signal_mask, dim3(1), dim3(64), 0, s, c->d_peer_flags, c->rank, c->epoch, c->nranks,
                         c->rank, mask, c->h_status);
      LHPC_HIP_TRY(hipGetLastError());
      LHPC_HIP_TRY(hipEventRecord(c->ev_in, s));  // u complete on the caller's stream
      LHPC_HIP_TRY(hipStreamWaitEvent(c->s_comm, c->ev_in, 0));
      hipLaunchKernelGGL(k_p2p_wait_mask, dim3(1), dim3(64), 0, c->s_comm, c->flags, 0, c->epoch, c->nranks, c->rank,
                         mask, c->h_status);
      LHPC_HIP_TRY(hipGetLastError());
      // plane 0 → the lower neighbour's plane nzl_lo (its upper ghost), plane
      // nzl − 1 → the upper neighbour's plane −1 (its lower ghost)
      HaloPut h{};
      int nt = 0;
      auto add = [&](int peer, const float *src, int64_t dst_off) {
        h.src[nt] = reinterpret_cast<const unsigned char *>(src);
        h.dst[nt] = static_cast<unsigned char *>(w->peer_buf[static_cast<size_t>(peer)]) + dst_off;
        h.bytes[nt] = pb;
        h.peer[nt] = peer;
        h.vec[nt] = (reinterpret_cast<uintptr_t>(h.src[nt]) | reinterpret_cast<uintptr_t>(h.dst[nt]) |
                     static_cast<uintptr_t>(pb)) % 16 == 0;
        ++nt;
      };
      if (lo) add(c->rank - 1, plane(0), (nzl_lo + ghost) * pb);
      if (hi) add(c->rank + 1, plane(nzl - 1), (ghost - 1) * pb);
      const unsigned bx = static_cast<unsigned>(std::min<int64_t>(32, (pb / 16 + 255) / 256 + 1));
      hipLaunchKernelGGL(k_p2p_halo_put, dim3(bx, static_cast<unsigned>(nt)), dim3(256), 0, c->s_comm, h, c->h_status,
                         c->flags, c->d_peer_flags, c->nranks, c->rank, c->epoch * 64u + 1u);
      LHPC_HIP_TRY(hipGetLastError());
      LHPC_HIP_TRY(hipEventRecord(c->ev_halo, c->s_comm));  // this rank's puts issued (u read)
    } else if (halo) {
      lhpc::RocTxRange rh("lhpc_dist_stencil7_f32: halo exchange");
      LHPC_HIP_TRY(hipEventRecord(c->ev_in, s));  // u complete on the caller's stream
      LHPC_HIP_TRY(hipStreamWaitEvent(c->s_comm, c->ev_in, 0));
      LHPC_NCCL_TRY(ncclGroupStart());
      if (lo) {
        LHPC_NCCL_TRY(ncclSend(plane(0), static_cast<size_t>(P), ncclFloat32, c->rank - 1, c->comm, c->s_comm));
        LHPC_NCCL_TRY(ncclRecv(plane(-1), static_cast<size_t>(P), ncclFloat32, c->rank - 1, c->comm, c->s_comm));
      }
      if (hi) {
        LHPC_NCCL_TRY(ncclSend(plane(nzl - 1), static_cast<size_t>(P), ncclFloat32, c->rank + 1, c->comm, c->s_comm));
        LHPC_NCCL_TRY(ncclRecv(plane(nzl), static_cast<size_t>(P), ncclFloat32, c->rank + 1, c->comm, c->s_comm));
      }
      LHPC_NCCL_TRY(ncclGroupEnd());
      LHPC_HIP_TRY(hipEventRecord(c->ev_halo, c->s_comm));
    }
    // interior planes need no halo: they run while the planes travel
    int st = LHPC_OK;
    if (nzl > 2) st = lhpc_stencil7_f32_planes(u, out, nzl, ny, nx, ghost, c0, c1, 1, nzl - 1, stream);
    if (st == LHPC_OK && halo) {
      if (w) {  // the neighbours' planes landed (DONE), stale L2 lines dropped
        hipLaunchKernelGGL(k_p2p_wait_acquire, dim3(kP2pAcqBlocks), dim3(64), 0, s, c->flags, c->nranks,
                           c->epoch * 64u + 1u, c->nranks, c->rank, c->h_status, mask);
        st = static_cast<int>(hipGetLastError());
      }
      // RCCL: the received planes; P2P: this rank's own puts, which read u's
      // boundary planes, end before the caller's next step writes them
      if (st == LHPC_OK) st = static_cast<int>(hipStreamWaitEvent(s, c->ev_halo, 0));
    }
    if (st == LHPC_OK) st = lhpc_stencil7_f32_planes(u, out, nzl, ny, nx, ghost, c0, c1, 0, 1, stream);
    if (st == LHPC_OK && nzl > 1)
      st = lhpc_stencil7_f32_planes(u, out, nzl, ny, nx, ghost, c0, c1, nzl - 1, nzl, stream);
    return st;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_dist_stencil7_f32(lhpc_dist_comm *c, float *u, float *out, int64_t nzl, int64_t ny,
                                      int64_t nx, int64_t ghost, float c0, float c1, void *stream) {
  try {
    return lhpc_dist_stencil7_f32_x(c, u, out, nzl, ny, nx, ghost, c0, c1, LHPC_DIST_EXCHANGE_AUTO, stream);
  } LHPC_ABI_CATCH
}
