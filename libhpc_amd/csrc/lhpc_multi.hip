// lhpc_multi.hip — row-block shares of a distributed SpMV, and the
// single-process multi-device plan (SURVEY §8b "Threading": "a multi-device
// plan internally does hipSetDevice per device and uses one stream and one
// RCCL comm per device").
//
// The reference has no multi-device code.  Its callers are
// single-process C++ programs holding their arrays as globals
// (tests/test_hpc_benchmark/test_hpc_benchmark.cpp:32-33); this plan lets
// such a caller reach every GPU of the node through the drop-in
// lhpc_spmv_plan_create(…, device_ids, n_devices, …) without becoming a
// launcher of one process per GPU.
//
//   shares   rows cut into D·K nnz-balanced blocks (lhpc_csr_partition_rows
//            with D·K parts), block b = k·D + d is device d's chunk k — the
//            same interleaved split as the one-process-per-GPU lhpc_dist_*
//            path, and the same local plans (LocalPlans: one row-range XTILE
//            plan over a device's K blocks, x staged once per call).
//   replica  lhpc_spmv_multi(plan, x[D], y[D], streams[D]): every device
//            holds full x and y; each reduces its chunk k straight into its
//            y, then its comm stream stores the block into every other
//            device's y (peer stores over xGMI; or RCCL group all-gathers,
//            ncclCommInitAll over distinct devices) while chunk k+1 is
//            reduced — the chunked copy/compute pipeline of the reference's
//            lib/gpu/transfer_overlap_testsuite/src/cuda_tut_transfer_overlap.cu:41-142
//            with an exchange in place of the copy.  All ordering between the
//            devices is HIP events issued by the one host thread: READY (this
//            device's y may be overwritten: recorded on its stream before any
//            push is issued), per-chunk push events, and a system-scope
//            acquire on every XCD of a device after its peers' stores landed
//            (they bypassed its L2s).
//   home     lhpc_spmv(plan, x, y, 1, stream): x and y on device_ids[0]; x is
//            copied to the other devices' plan-owned replicas, every device
//            computes its blocks, and the blocks come back into y.  With host
//            buffers (on_device 0) x goes host → every device and the blocks
//            device → host y.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "lhpc_common.hpp"
#include "lhpc_rccl.hpp"
#include "lhpc_spmv_impl.hpp"

// ------------------------------------------------------------ local plans
namespace lhpc {

int local_plans_create(LocalPlans &lp, int dtype, int64_t n_cols, int K, const int64_t *ls, const void *row_ptr,
                       int row_ptr_bits, const int32_t *col_idx, const void *val, int device, unsigned flags,
                       const lhpc_options &o) {
  lp = LocalPlans{};
  lp.K = K;
  lhpc_options lo = o;
  lo.multi_force = 0;  // the local plans are single-device plans
  // ranges are gathered and reduced one after the other (local_plans_chunk),
  // so cache-sized ranges can share one xg ring
  if (lo.xtile_ring == 0) lo.xtile_ring = 2;
  lp.ls.assign(ls, ls + K + 1);
  const RowPtrView rp{row_ptr, row_ptr_bits};
  const int64_t n_local = ls[K];
  const int64_t nnz_local = rp[n_local];
  const size_t tsz = dtype == LHPC_F64 ? 8 : 4;
  // splits at the starts of non-empty blocks after the first row
  std::vector<int64_t> splits;
  lp.range_of.assign(static_cast<size_t>(K), -1);
  int nrange = 0;
  for (int k = 0; k < K; ++k) {
    if (ls[k + 1] == ls[k]) continue;
    if (ls[k] > 0) splits.push_back(ls[k]);
    lp.range_of[k] = nrange++;
  }
  int st = LHPC_OK;
  if (!splits.empty())
    st = lhpc_spmv_plan_create_opts(&lp.split, dtype, n_local, n_cols, nnz_local, row_ptr, row_ptr_bits, col_idx,
                                    val, &device, 1, flags, static_cast<int>(splits.size()), splits.data(), &lo);
  if (splits.empty() || st == LHPC_ERR_UNSUPPORTED) {
    // one plan per non-empty block (the matrix does not select XTILE, or a
    // single block)
    lp.split = nullptr;
    st = LHPC_OK;
    lp.block_plan.assign(static_cast<size_t>(K), nullptr);
    std::vector<int64_t> lrp;
    for (int k = 0; k < K && st == LHPC_OK; ++k) {
      const int64_t r0 = ls[k], r1 = ls[k + 1];
      if (r1 == r0) continue;
      const int64_t e0 = rp[r0], e1 = rp[r1];
      lrp.resize(static_cast<size_t>(r1 - r0 + 1));
      for (int64_t i = r0; i <= r1; ++i) lrp[static_cast<size_t>(i - r0)] = rp[i] - e0;
      st = lhpc_spmv_plan_create_opts(&lp.block_plan[k], dtype, r1 - r0, n_cols, e1 - e0, lrp.data(), 64,
                                      col_idx + e0, static_cast<const unsigned char *>(val) + e0 * tsz, &device, 1,
                                      flags, 0, nullptr, &lo);
    }
  }
  if (st != LHPC_OK) local_plans_destroy(lp);
  return st;
}

void local_plans_destroy(LocalPlans &lp) {
  if (lp.split) lhpc_spmv_plan_destroy(lp.split);
  for (auto *p : lp.block_plan)
    if (p) lhpc_spmv_plan_destroy(p);
  lp = LocalPlans{};
}

int local_plans_stage(const LocalPlans &lp, const void *x, hipStream_t s) {
  if (lp.split && !lp.range_gather()) return xtile_stage(lp.split, x, s);
  return LHPC_OK;
}

bool local_plans_column_parts(LocalPlans &lp, const int64_t *col_end, int n_parts) {
  if (!lp.split || lp.range_gather()) return false;
  return xtile_column_parts(lp.split, col_end, n_parts) == LHPC_OK;
}

int local_plans_stage_part(const LocalPlans &lp, const void *x, int j, hipStream_t s) {
  if (!lp.column_parts()) return LHPC_ERR_UNSUPPORTED;
  return xtile_stage_part(lp.split, x, j, s);
}

int local_plans_chunk(const LocalPlans &lp, const void *x, int k, void *yk, int &gathered, hipStream_t s) {
  const int r = lp.range_of[static_cast<size_t>(k)];
  if (r < 0) return LHPC_OK;  // empty block
  if (lp.split) {
    if (lp.range_gather())
      for (; gathered <= r; ++gathered) LHPC_TRY(xtile_range_gather(lp.split, x, gathered, s));
    return xtile_range(lp.split, r, yk, s);
  }
  return lhpc_spmv(lp.block_plan[static_cast<size_t>(k)], x, yk, 1, s);
}

void local_csr_from_global(LocalCsr &out, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz,
                           const int64_t *cuts, int nranks, int K, int rank) {
  out = LocalCsr{};
  out.ls.assign(static_cast<size_t>(K) + 1, 0);
  for (int k = 0; k < K; ++k) {
    const int64_t b = static_cast<int64_t>(k) * nranks + rank;
    out.ls[k + 1] = out.ls[k] + (cuts[b + 1] - cuts[b]);
  }
  out.rp.assign(static_cast<size_t>(out.ls[K]) + 1, 0);
  int64_t nnz = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t b = static_cast<int64_t>(k) * nranks + rank, r0 = cuts[b], r1 = cuts[b + 1];
    for (int64_t r = r0; r < r1; ++r) out.rp[static_cast<size_t>(out.ls[k] + r - r0 + 1)] = nnz + rp[r + 1] - rp[r0];
    nnz += rp[r1] - rp[r0];
  }
  // one non-empty block: the caller's col/val at its offset, no copy
  int nonempty = 0, only = -1;
  for (int k = 0; k < K; ++k)
    if (out.ls[k + 1] > out.ls[k]) ++nonempty, only = k;
  if (nonempty <= 1) {
    const int64_t e0 = only < 0 ? 0 : rp[cuts[static_cast<int64_t>(only) * nranks + rank]];
    out.colp = col_idx + e0;
    out.valp = static_cast<const unsigned char *>(val) + e0 * static_cast<int64_t>(tsz);
    return;
  }
  out.col.resize(static_cast<size_t>(nnz));
  out.val.resize(static_cast<size_t>(nnz) * tsz);
  int64_t at = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t b = static_cast<int64_t>(k) * nranks + rank, e0 = rp[cuts[b]], e1 = rp[cuts[b + 1]];
    if (e1 > e0) {
      std::memcpy(out.col.data() + at, col_idx + e0, static_cast<size_t>(e1 - e0) * 4);
      std::memcpy(out.val.data() + at * tsz, static_cast<const unsigned char *>(val) + e0 * tsz,
                  static_cast<size_t>(e1 - e0) * tsz);
    }
    at += e1 - e0;
  }
  out.colp = out.col.data();
  out.valp = out.val.data();
}

}  // namespace lhpc

// ------------------------------------------------------ multi-device plan
#define LHPC_NCCL_TRY(expr)                                                \
  do {                                                                     \
    ncclResult_t _r = (expr);                                              \
    if (_r != ncclSuccess) return LHPC_RCCL_STATUS_BASE + static_cast<int>(_r); \
  } while (0)

constexpr int kMultiMaxDevices = 16;

struct MultiDev {
  int device = 0;
  hipStream_t s = nullptr;       // plan-owned compute stream (home / host calls, NULL streams)
  hipStream_t s_comm = nullptr;  // exchange stream
  lhpc::LocalPlans lp;
  void *d_x = nullptr, *d_y = nullptr;  // plan-owned full replicas (home / host calls)
  std::vector<hipEvent_t> ev_red, ev_push;  // [K] chunk k reduced / pushed to the peers
  hipEvent_t ev_ready = nullptr, ev_done = nullptr;
  ncclComm_t comm = nullptr;
  int cus = 256;
};

struct lhpc_multi {
  int D = 1, K = 1, dtype = LHPC_F32;
  int64_t n_rows = 0, n_cols = 0;
  int exchange = LHPC_DIST_EXCHANGE_P2P;  // resolved: P2P (peer stores) or RCCL
  bool distinct = true;                   // no device listed twice
  std::vector<int64_t> cuts;              // D·K + 1
  std::vector<lhpc_dist_xfer> sched;      // RCCL schedule of device 0's view (root/offsets are global)
  std::vector<std::vector<lhpc_dist_xfer>> sched_dev;  // per device (send offsets differ)
  // their RCCL calls (lhpc_rccl.hpp; one per schedule entry, so first[] indexes
  // both).  Each chunk's calls of all devices go in one outer group: one
  // process drives every communicator
  std::vector<std::vector<lhpc_rccl_call>> calls_dev;
  std::vector<int64_t> first;             // chunk k's entries [first[k], first[k+1])
  MultiDev dev[kMultiMaxDevices];
  hipEvent_t ev_start = nullptr;          // home calls: recorded on the caller's stream
};

namespace {
using namespace lhpc;

struct PeerPtrs {
  void *p[kMultiMaxDevices];
};

// bytes [o0, o1) of `src` into the same bytes of every target in `dst`
// (blockIdx.y = target; o0/o1 multiples of 4): 16-B stores over the
// interior both sides share a 16-B phase on, words elsewhere.  The stores
// cross xGMI when the target sits on another device (peer access enabled)
__global__ __launch_bounds__(256) void k_multi_push(PeerPtrs dst, const unsigned char *src, int64_t o0, int64_t o1) {
  unsigned char *d = static_cast<unsigned char *>(dst.p[blockIdx.y]);
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x, T = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const uintptr_t sb = reinterpret_cast<uintptr_t>(src), db = reinterpret_cast<uintptr_t>(d);
  int64_t a0 = static_cast<int64_t>(((sb + o0 + 15) & ~uintptr_t{15}) - sb);
  int64_t a1 = static_cast<int64_t>(((sb + o1) & ~uintptr_t{15}) - sb);
  if (((sb ^ db) & 15) != 0 || a0 >= a1) a0 = a1 = o1;  // other phase: words only
  for (int64_t i = o0 + 4 * t; i < a0; i += 4 * T)
    *reinterpret_cast<uint32_t *>(d + i) = *reinterpret_cast<const uint32_t *>(src + i);
  for (int64_t i = a0 + 16 * t; i < a1; i += 16 * T)
    *reinterpret_cast<uint4 *>(d + i) = *reinterpret_cast<const uint4 *>(src + i);
  for (int64_t i = a1 + 4 * t; i < o1; i += 4 * T)
    *reinterpret_cast<uint32_t *>(d + i) = *reinterpret_cast<const uint32_t *>(src + i);
  __threadfence_system();
}

// after peers' stores into this device's y: a system-scope acquire on every
// XCD (one block per CU, dealt round-robin over the XCDs), so no L2 keeps a
// stale line of y that the next call's gather would read as x
__global__ void k_multi_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

void multi_destroy(lhpc_multi *m) {
  if (!m) return;
  for (int d = 0; d < m->D; ++d) {
    MultiDev &v = m->dev[d];
    (void)hipSetDevice(v.device);
    if (v.s) (void)hipStreamSynchronize(v.s);
    if (v.s_comm) (void)hipStreamSynchronize(v.s_comm);
  }
  for (int d = 0; d < m->D; ++d) {
    MultiDev &v = m->dev[d];
    (void)hipSetDevice(v.device);
    local_plans_destroy(v.lp);
    if (v.d_x) (void)hipFree(v.d_x);
    if (v.d_y) (void)hipFree(v.d_y);
    for (hipEvent_t e : v.ev_red)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : v.ev_push)
      if (e) (void)hipEventDestroy(e);
    if (v.ev_ready) (void)hipEventDestroy(v.ev_ready);
    if (v.ev_done) (void)hipEventDestroy(v.ev_done);
    if (v.comm) (void)ncclCommDestroy(v.comm);
    if (v.s) (void)hipStreamDestroy(v.s);
    if (v.s_comm) (void)hipStreamDestroy(v.s_comm);
  }
  if (m->ev_start) {
    (void)hipSetDevice(m->dev[0].device);
    (void)hipEventDestroy(m->ev_start);
  }
  delete m;
}

size_t tsize(const lhpc_multi *m) { return m->dtype == LHPC_F64 ? 8 : 4; }

// chunk k: every device reduces its block into ys[d] and hands it to its
// comm stream, which delivers it to the devices `to` lists (P2P: peer
// stores; RCCL: the group all-gather of the schedule, every device)
int multi_chunks(lhpc_multi *m, const void *const *xs, void *const *ys, const hipStream_t *ss, bool all_to_all,
                 bool home_only) {
  const size_t tsz = tsize(m);
  const int D = m->D;
  std::vector<int> gathered(static_cast<size_t>(D), 0);
  // READY: every device's y may be overwritten once its stream reaches here
  for (int d = 0; d < D; ++d) {
    MultiDev &v = m->dev[d];
    LHPC_HIP_TRY(hipSetDevice(v.device));
    LHPC_HIP_TRY(hipEventRecord(v.ev_ready, ss[d]));
    LHPC_TRY(local_plans_stage(v.lp, xs[d], ss[d]));
  }
  const bool rccl = m->exchange == LHPC_DIST_EXCHANGE_RCCL && all_to_all;
  for (int k = 0; k < m->K; ++k) {
    for (int d = 0; d < D; ++d) {
      MultiDev &v = m->dev[d];
      LHPC_HIP_TRY(hipSetDevice(v.device));
      const int64_t b = static_cast<int64_t>(k) * D + d;
      void *yk = static_cast<unsigned char *>(ys[d]) + m->cuts[b] * tsz;
      LHPC_TRY(local_plans_chunk(v.lp, xs[d], k, yk, gathered[static_cast<size_t>(d)], ss[d]));
      if (D == 1 && !rccl) continue;
      LHPC_HIP_TRY(hipEventRecord(v.ev_red[k], ss[d]));
      LHPC_HIP_TRY(hipStreamWaitEvent(v.s_comm, v.ev_red[k], 0));
      if (rccl) continue;  // the group below
      const int64_t o0 = m->cuts[b] * static_cast<int64_t>(tsz), o1 = m->cuts[b + 1] * static_cast<int64_t>(tsz);
      PeerPtrs pp{};
      unsigned np = 0;
      for (int p = 0; p < D; ++p) {
        if (p == d || (home_only && p != 0)) continue;
        if (k == 0) LHPC_HIP_TRY(hipStreamWaitEvent(v.s_comm, m->dev[p].ev_ready, 0));
        pp.p[np++] = ys[p];
      }
      if (np > 0 && o1 > o0) {
        lhpc::RocTxRange rb("lhpc_spmv_multi: y chunk push");
        const int64_t vec = (o1 - o0) / 16 + 1;
        const unsigned bx = static_cast<unsigned>(std::min<int64_t>(64, (vec + 255) / 256));
        hipLaunchKernelGGL(k_multi_push, dim3(bx, np), dim3(256), 0, v.s_comm, pp,
                           static_cast<const unsigned char *>(ys[d]), o0, o1);
        LHPC_HIP_TRY(hipGetLastError());
      }
      LHPC_HIP_TRY(hipEventRecord(v.ev_push[k], v.s_comm));
    }
    if (rccl) {
      // chunk k's all-gather (or broadcasts) as one group over the devices
      LHPC_NCCL_TRY(ncclGroupStart());
      for (int d = 0; d < D; ++d) {
        MultiDev &v = m->dev[d];
        unsigned char *yb = static_cast<unsigned char *>(ys[d]);
        const auto &cd = m->calls_dev[static_cast<size_t>(d)];  // lhpc_rccl.hpp records, as lhpc_dist_rccl_calls
        for (int64_t e = m->first[k]; e < m->first[k + 1]; ++e) {
          const ncclResult_t r = rccl_issue(cd[static_cast<size_t>(e)], yb, v.comm, v.s_comm);
          if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return LHPC_RCCL_STATUS_BASE + static_cast<int>(r);
          }
        }
      }
      LHPC_NCCL_TRY(ncclGroupEnd());
      for (int d = 0; d < D; ++d) {
        LHPC_HIP_TRY(hipSetDevice(m->dev[d].device));
        LHPC_HIP_TRY(hipEventRecord(m->dev[d].ev_push[k], m->dev[d].s_comm));
      }
    }
  }
  if (D == 1 && !rccl) return LHPC_OK;
  // every device's stream waits for what was pushed into its y, then drops
  // stale L2 lines of y (peer stores bypassed its L2s).  It also waits for
  // its OWN pushes (they read ys[d]): a write to ys[d] queued on ss[d] after
  // the call — a user kernel, or the next call's reduce, which waits only on
  // READY — must not race the push that copies ys[d]'s blocks to the peers
  for (int d = 0; d < D; ++d) {
    MultiDev &v = m->dev[d];
    LHPC_HIP_TRY(hipSetDevice(v.device));
    if (home_only && d != 0) {
      if (!rccl) LHPC_HIP_TRY(hipStreamWaitEvent(ss[d], v.ev_push[m->K - 1], 0));  // s_comm is in order
      continue;
    }
    bool remote = rccl;
    for (int p = 0; p < D; ++p) {
      if (p == d && !rccl) {
        LHPC_HIP_TRY(hipStreamWaitEvent(ss[d], v.ev_push[m->K - 1], 0));
        continue;
      }
      for (int k = 0; k < m->K; ++k) LHPC_HIP_TRY(hipStreamWaitEvent(ss[d], m->dev[p].ev_push[k], 0));
      if (m->dev[p].device != v.device) remote = true;
    }
    if (remote) {
      hipLaunchKernelGGL(k_multi_acquire, dim3(static_cast<unsigned>(v.cus)), dim3(64), 0, ss[d]);
      LHPC_HIP_TRY(hipGetLastError());
    }
  }
  return LHPC_OK;
}

}  // namespace

namespace lhpc {

int multi_create(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, const int *device_ids,
                 int n_devices, unsigned flags) {
  const lhpc_options &o = p->opt;
  if (n_devices < 1 || n_devices > kMultiMaxDevices || !device_ids) return LHPC_ERR_INVALID_ARG;
  auto *m = new (std::nothrow) lhpc_multi();
  if (!m) return LHPC_ERR_ALLOC;
  p->multi = m;
  m->D = n_devices;
  m->K = o.multi_chunks > 0 ? o.multi_chunks : 2;
  if (m->K > 64) return LHPC_ERR_INVALID_ARG;
  m->dtype = p->dtype;
  m->n_rows = p->n_rows;
  m->n_cols = p->n_cols;
  const int D = m->D, K = m->K;
  for (int d = 0; d < D; ++d)
    for (int e = 0; e < d; ++e)
      if (device_ids[d] == device_ids[e]) m->distinct = false;
  const int xo = o.multi_exchange;
  if (xo == LHPC_DIST_EXCHANGE_RCCL) {
    if (!m->distinct) return LHPC_ERR_UNSUPPORTED;  // RCCL needs one rank per device
    m->exchange = LHPC_DIST_EXCHANGE_RCCL;
  } else if (xo == LHPC_DIST_EXCHANGE_AUTO || xo == LHPC_DIST_EXCHANGE_P2P) {
    m->exchange = LHPC_DIST_EXCHANGE_P2P;
  } else {
    return LHPC_ERR_INVALID_ARG;
  }
  const size_t tsz = p->dtype == LHPC_F64 ? 8 : 4;
  // nnz-balanced interleaved blocks (block k·D + d: device d's chunk k)
  m->cuts.assign(static_cast<size_t>(D) * K + 1, 0);
  LHPC_TRY(lhpc_csr_partition_rows(rp.p, rp.bits, p->n_rows, D * K, m->cuts.data()));
  // per-device RCCL schedules (lhpc_dist_exchange_schedule): the same calls
  // on every device, send offsets its own
  if (m->exchange == LHPC_DIST_EXCHANGE_RCCL) {
    m->sched_dev.resize(static_cast<size_t>(D));
    for (int d = 0; d < D; ++d) {
      std::vector<lhpc_dist_xfer> v(static_cast<size_t>(D) * K + 1);
      int64_t n = 0;
      LHPC_TRY(lhpc_dist_exchange_schedule(m->cuts.data(), D, K, d, LHPC_DIST_EXCHANGE_RCCL, o.dist_broadcast,
                                           v.data(), static_cast<int64_t>(v.size()), &n));
      v.resize(static_cast<size_t>(n));
      m->sched_dev[static_cast<size_t>(d)] = v;
      m->calls_dev.emplace_back();
      rccl_calls_of(v.data(), n, p->dtype, m->calls_dev.back());
    }
    m->first.assign(static_cast<size_t>(K) + 1, 0);
    const auto &s0 = m->sched_dev[0];
    for (int k = 0, e = 0; k <= K; ++k) {
      while (e < static_cast<int>(s0.size()) && s0[static_cast<size_t>(e)].chunk < k) ++e;
      m->first[static_cast<size_t>(k)] = e;
    }
  }
  for (int d = 0; d < D; ++d) {
    MultiDev &v = m->dev[d];
    v.device = device_ids[d];
    LHPC_HIP_TRY(hipSetDevice(v.device));
    hipDeviceProp_t prop;
    LHPC_HIP_TRY(hipGetDeviceProperties(&prop, v.device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LHPC_ERR_NO_DEVICE;
    v.cus = prop.multiProcessorCount >= 8 ? prop.multiProcessorCount : 256;
    LHPC_HIP_TRY(hipStreamCreateWithFlags(&v.s, hipStreamNonBlocking));
    LHPC_HIP_TRY(hipStreamCreateWithFlags(&v.s_comm, hipStreamNonBlocking));
    v.ev_red.assign(static_cast<size_t>(K), nullptr);
    v.ev_push.assign(static_cast<size_t>(K), nullptr);
    for (auto &e : v.ev_red) LHPC_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto &e : v.ev_push) LHPC_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    LHPC_HIP_TRY(hipEventCreateWithFlags(&v.ev_ready, hipEventDisableTiming));
    LHPC_HIP_TRY(hipEventCreateWithFlags(&v.ev_done, hipEventDisableTiming));
    // peer access to every other device listed (stores over xGMI)
    for (int e = 0; e < D; ++e) {
      if (device_ids[e] == v.device) continue;
      int can = 0;
      LHPC_HIP_TRY(hipDeviceCanAccessPeer(&can, v.device, device_ids[e]));
      if (!can) return LHPC_ERR_UNSUPPORTED;
      const hipError_t he = hipDeviceEnablePeerAccess(device_ids[e], 0);
      if (he == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      else if (he != hipSuccess) return static_cast<int>(he);
    }
    LocalCsr lc;
    local_csr_from_global(lc, rp, col_idx, val, tsz, m->cuts.data(), D, K, d);
    LHPC_TRY(local_plans_create(v.lp, p->dtype, p->n_cols, K, lc.ls.data(), lc.rp.data(), 64, lc.colp, lc.valp,
                                v.device, flags, o));
    LHPC_TRY(dmalloc(&v.d_x, static_cast<size_t>(std::max<int64_t>(p->n_cols, 1)) * tsz, p->bytes));
    LHPC_TRY(dmalloc(&v.d_y, static_cast<size_t>(std::max<int64_t>(p->n_rows, 1)) * tsz, p->bytes));
    for (const lhpc_spmv_plan *q : v.lp.block_plan)
      if (q) p->bytes += q->bytes;
    if (v.lp.split) p->bytes += v.lp.split->bytes;
  }
  if (m->exchange == LHPC_DIST_EXCHANGE_RCCL) {
    std::vector<ncclComm_t> comms(static_cast<size_t>(D));
    LHPC_NCCL_TRY(ncclCommInitAll(comms.data(), D, device_ids));
    for (int d = 0; d < D; ++d) m->dev[d].comm = comms[static_cast<size_t>(d)];
  }
  LHPC_HIP_TRY(hipSetDevice(m->dev[0].device));
  LHPC_HIP_TRY(hipEventCreateWithFlags(&m->ev_start, hipEventDisableTiming));
  // what the single-device fields report: device 0's local plan family
  const lhpc_spmv_plan *q0 = m->dev[0].lp.split;
  for (const lhpc_spmv_plan *q : m->dev[0].lp.block_plan)
    if (!q0 && q) q0 = q;
  p->kernel = q0 ? q0->kernel : LHPC_KERNEL_ADAPTIVE;
  p->S = q0 ? q0->S : 0;
  p->xs_width = q0 ? q0->xs_width : 0;
  p->device = m->dev[0].device;
  return LHPC_OK;
}

void multi_free(lhpc_spmv_plan *p) {
  multi_destroy(p->multi);
  p->multi = nullptr;
}

// lhpc_spmv on a multi-device plan (x, y on device_ids[0], or host buffers)
int multi_home(lhpc_spmv_plan *p, const void *x, void *y, int on_device, hipStream_t s) {
  lhpc_multi *m = p->multi;
  const size_t tsz = tsize(m);
  const int D = m->D;
  const size_t xb = static_cast<size_t>(m->n_cols) * tsz;
  std::vector<const void *> xs(static_cast<size_t>(D));
  std::vector<void *> ys(static_cast<size_t>(D));
  std::vector<hipStream_t> ss(static_cast<size_t>(D));
  if (!on_device) {
    // host x → every device's replica (synchronous copies: no asynchronous
    // copy touches pageable host memory)
    for (int d = 0; d < D; ++d) {
      MultiDev &v = m->dev[d];
      LHPC_HIP_TRY(hipSetDevice(v.device));
      if (xb) LHPC_HIP_TRY(hipMemcpy(v.d_x, x, xb, hipMemcpyHostToDevice));
      xs[d] = v.d_x;
      ys[d] = v.d_y;
      ss[d] = v.s;
    }
    LHPC_TRY(multi_chunks(m, xs.data(), ys.data(), ss.data(), false, false));
    for (int d = 0; d < D; ++d) {
      MultiDev &v = m->dev[d];
      LHPC_HIP_TRY(hipSetDevice(v.device));
      LHPC_HIP_TRY(hipStreamSynchronize(v.s));
      for (int k = 0; k < m->K; ++k) {
        const int64_t b = static_cast<int64_t>(k) * D + d, r0 = m->cuts[b], r1 = m->cuts[b + 1];
        if (r1 > r0)
          LHPC_HIP_TRY(hipMemcpy(static_cast<unsigned char *>(y) + r0 * tsz, static_cast<unsigned char *>(v.d_y) + r0 * tsz,
                                 static_cast<size_t>(r1 - r0) * tsz, hipMemcpyDeviceToHost));
      }
    }
    LHPC_HIP_TRY(hipSetDevice(m->dev[0].device));
    return LHPC_OK;
  }
  // device buffers on device_ids[0]: the other devices start after the
  // caller's stream reached this call, copy x into their replicas, and their
  // blocks are stored into y (home_only push); the caller's stream then
  // waits for every device
  LHPC_HIP_TRY(hipSetDevice(m->dev[0].device));
  LHPC_HIP_TRY(hipEventRecord(m->ev_start, s));
  for (int d = 0; d < D; ++d) {
    MultiDev &v = m->dev[d];
    if (d == 0) {
      xs[0] = x;
      ys[0] = y;
      ss[0] = s;
      continue;
    }
    LHPC_HIP_TRY(hipSetDevice(v.device));
    LHPC_HIP_TRY(hipStreamWaitEvent(v.s, m->ev_start, 0));
    if (xb) LHPC_HIP_TRY(hipMemcpyPeerAsync(v.d_x, v.device, x, m->dev[0].device, xb, v.s));
    xs[d] = v.d_x;
    ys[d] = v.d_y;
    ss[d] = v.s;
  }
  LHPC_TRY(multi_chunks(m, xs.data(), ys.data(), ss.data(), false, true));
  // y complete on `s` once every other device's stream is done (its blocks
  // were pushed by its comm stream, which the push events already cover)
  for (int d = 1; d < D; ++d) {
    MultiDev &v = m->dev[d];
    LHPC_HIP_TRY(hipSetDevice(v.device));
    LHPC_HIP_TRY(hipEventRecord(v.ev_done, v.s));
    LHPC_HIP_TRY(hipSetDevice(m->dev[0].device));
    LHPC_HIP_TRY(hipStreamWaitEvent(s, v.ev_done, 0));
  }
  LHPC_HIP_TRY(hipSetDevice(m->dev[0].device));
  return LHPC_OK;
}

}  // namespace lhpc

using namespace lhpc;

extern "C" int lhpc_spmv_multi(lhpc_spmv_plan *p, const void *const *x, void *const *y, void *const *streams) {
  try {
    if (!p || !p->multi || !x || !y) return LHPC_ERR_INVALID_ARG;
    lhpc_multi *m = p->multi;
    const int D = m->D;
    std::vector<const void *> xs(static_cast<size_t>(D));
    std::vector<void *> ys(static_cast<size_t>(D));
    std::vector<hipStream_t> ss(static_cast<size_t>(D));
    for (int d = 0; d < D; ++d) {
      if ((m->n_cols > 0 && !x[d]) || (m->n_rows > 0 && !y[d]) || (x[d] == y[d] && m->n_rows > 0))
        return LHPC_ERR_INVALID_ARG;
      for (int e = 0; e < d; ++e)
        if (y[e] == y[d] && m->n_rows > 0) return LHPC_ERR_INVALID_ARG;  // one y replica per device
      xs[d] = x[d];
      ys[d] = y[d];
      ss[d] = streams ? static_cast<hipStream_t>(streams[d]) : m->dev[d].s;
    }
    RocTxRange rx("lhpc_spmv_multi");
    const int st = multi_chunks(m, xs.data(), ys.data(), ss.data(), true, false);
    (void)hipSetDevice(m->dev[0].device);
    return st;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_spmv_plan_multi_info(const lhpc_spmv_plan *p, int *n_devices, int *chunks, int *exchange,
                                         int *device_ids, int64_t *cuts) {
  try {
    if (!p) return LHPC_ERR_INVALID_ARG;
    const lhpc_multi *m = p->multi;
    const int D = m ? m->D : 1, K = m ? m->K : 1;
    if (n_devices) *n_devices = D;
    if (chunks) *chunks = K;
    if (exchange) *exchange = m ? m->exchange : LHPC_DIST_EXCHANGE_NONE;
    if (device_ids)
      for (int d = 0; d < D; ++d) device_ids[d] = m ? m->dev[d].device : p->device;
    if (cuts) {
      if (m) std::copy(m->cuts.begin(), m->cuts.end(), cuts);
      else cuts[0] = 0, cuts[1] = p->n_rows;
    }
    return LHPC_OK;
  } LHPC_ABI_CATCH
}
