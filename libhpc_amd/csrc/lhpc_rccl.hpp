// lhpc_rccl.hpp — the RCCL calls of the y exchange, from the exchange
// schedule (lhpc_dist_exchange_schedule), as plain argument records
// (include/lhpc.h lhpc_rccl_call).  lhpc_dist.hip (one process per rank) and
// lhpc_multi.hip (one process, one communicator per device) issue their
// collectives only through rccl_calls_of + rccl_issue, and
// lhpc_dist_rccl_calls exports the same records to the CPU tests
// (tests/test_dist.py: matching collectives, in-place all-gather slots,
// broadcast roots, emulated end to end for N = 8, K = 1/2/4).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <vector>

#include "../../include/lhpc.h"

namespace lhpc {

inline ncclDataType_t rccl_dtype(int dtype) { return dtype == LHPC_F64 ? ncclFloat64 : ncclFloat32; }

// the calls of schedule entries x[0, n) (one rank's view, RCCL exchange);
// entries flagged `group` are bracketed per chunk (ncclGroupStart before the
// chunk's first, ncclGroupEnd after its last)
inline void rccl_calls_of(const lhpc_dist_xfer *x, int64_t n, int dtype, std::vector<lhpc_rccl_call> &out) {
  const int64_t tsz = dtype == LHPC_F64 ? 8 : 4;
  for (int64_t e = 0; e < n; ++e) {
    const lhpc_dist_xfer &t = x[e];
    lhpc_rccl_call c{};
    c.chunk = t.chunk;
    c.datatype = static_cast<int32_t>(rccl_dtype(dtype));
    c.count = t.count;
    c.recv_byte_offset = t.offset * tsz;
    if (t.kind == LHPC_XFER_ALLGATHER) {
      c.op = LHPC_RCCL_ALLGATHER;
      c.root = -1;
      c.send_byte_offset = t.send_offset * tsz;  // in place: recv + rank·count
    } else {
      c.op = LHPC_RCCL_BROADCAST;
      c.root = t.root;
      c.send_byte_offset = t.offset * tsz;  // in place on every rank (only the root's is read)
    }
    const bool first = e == 0 || x[e - 1].chunk != t.chunk, last = e + 1 == n || x[e + 1].chunk != t.chunk;
    c.group_begin = t.group && first ? 1 : 0;
    c.group_end = t.group && last ? 1 : 0;
    out.push_back(c);
  }
}

// one call on y (the group brackets are the caller's: rccl_issue_list)
inline ncclResult_t rccl_issue(const lhpc_rccl_call &c, unsigned char *y, ncclComm_t comm, hipStream_t s) {
  const auto dt = static_cast<ncclDataType_t>(c.datatype);
  if (c.op == LHPC_RCCL_ALLGATHER)
    return ncclAllGather(y + c.send_byte_offset, y + c.recv_byte_offset, static_cast<size_t>(c.count), dt, comm, s);
  return ncclBroadcast(y + c.send_byte_offset, y + c.recv_byte_offset, static_cast<size_t>(c.count), dt, c.root, comm,
                       s);
}

// calls [c0, c1) with their group brackets (lhpc_dist_spmv's chunk exchange)
inline int rccl_issue_list(const lhpc_rccl_call *c, int64_t c0, int64_t c1, unsigned char *y, ncclComm_t comm,
                           hipStream_t s) {
  bool open = false;
  for (int64_t i = c0; i < c1; ++i) {
    if (c[i].group_begin) {
      const ncclResult_t r = ncclGroupStart();
      if (r != ncclSuccess) return LHPC_RCCL_STATUS_BASE + static_cast<int>(r);
      open = true;
    }
    const ncclResult_t r = rccl_issue(c[i], y, comm, s);
    if (r != ncclSuccess) {
      if (open) (void)ncclGroupEnd();
      return LHPC_RCCL_STATUS_BASE + static_cast<int>(r);
    }
    if (c[i].group_end) {
      open = false;
      const ncclResult_t g = ncclGroupEnd();
      if (g != ncclSuccess) return LHPC_RCCL_STATUS_BASE + static_cast<int>(g);
    }
  }
  if (open) {
    const ncclResult_t g = ncclGroupEnd();
    if (g != ncclSuccess) return LHPC_RCCL_STATUS_BASE + static_cast<int>(g);
  }
  return LHPC_OK;
}

}  // namespace lhpc
