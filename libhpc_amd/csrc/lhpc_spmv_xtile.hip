// lhpc_spmv_xtile.hip — XTILE: CSR SpMV with x tiles in LDS (DESIGN.md §4
// XTILE; layout: lhpc_plan.hpp XtileHost).  The default for matrices whose
// x does not fit L2 and whose gathers have no locality (C2–C4): every x read
// is an LDS read, every HBM access a coalesced stream.
//   gather  one workgroup per (tile, piece): tile s of x (160 KB) in LDS, the
//           tile's nonzeros streamed as u16 column offsets; writes xg[g] =
//           x[col] in tile-stream order;
//   reduce  one workgroup per chunk of ≤ M CSR nonzeros: the chunk's S
//           segments of xg into LDS, a segmented scan of the products per
//           row in CSR order (fp64), the owned rows' y stored coalesced;
//   fixup   rows cut by a chunk end: their fp64 pieces added in chunk order.
// Numerics: fp32 products are exact in fp64 and summed in fp64, rounded once
// at the store; fp64 products are rounded once, as in the reference loop.
// Dyadic inputs are bit-exact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lhpc_plan.hpp"
#include "lhpc_spmv_impl.hpp"

namespace lhpc {
namespace {

constexpr int kXtGatherBlock = 1024;  // gather: 16 waves per CU, one tile of x in LDS
constexpr int kXtFixBlock = 256;      // fix-up
template <typename T> struct XtTile;
template <> struct XtTile<float> { static constexpr int W = 40960; };   // 160 KB
template <> struct XtTile<double> { static constexpr int W = 20480; };  // 160 KB

// gather: block b streams pieces[3b..3b+1] of tile pieces[3b+2]; 8 nonzeros
// per thread and step (one 16-B col16 load, 8 LDS gathers, 8 contiguous xg
// stores), U steps in flight.  Piece bounds are multiples of 8.  The first
// col16 step does not depend on the tile, so it is issued under the tile load.
// (A fused form that also streamed val in tile order and wrote val·x[col]
// was slower: C2 603 → 621 µs, C3 1141 → 1736 µs)
#ifdef LHPC_XT_PROBE_GVAL
// timing-only probe (wrong results): the gather also streams one T per entry
// (from the plan's val, index masked into range) and writes val·x
#define LHPC_GVAL_PARAM , const T *__restrict__ vg, int64_t vmask
#else
#define LHPC_GVAL_PARAM
#endif
// pext (xg ring plans, lhpc_plan.hpp xtile_ring_pieces): {delta, flags} per
// piece — every xg store lands at stream position + delta, and thread 0 /
// thread 1 also gather the group before the piece / at its end (flags bit 0
// / 1: an 8-entry group two ranges share, col16 unpermuted, stored as 8
// contiguous entries); nullptr: delta 0, no extra groups.
template <typename T, int U, bool NT = false>
__global__ __launch_bounds__(kXtGatherBlock) void k_xtile_gather(
    const int32_t *__restrict__ pieces, const uint16_t *__restrict__ col16,
    const T *__restrict__ x, int64_t n_cols, int tw, T *__restrict__ xg,
    const int32_t *__restrict__ pext LHPC_GVAL_PARAM) {
  constexpr int W = XtTile<T>::W;  // LDS capacity; the plan's tile width tw ≤ W
  __shared__ T xt[W];
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int g0 = pieces[3 * blockIdx.x], g1 = pieces[3 * blockIdx.x + 1];
  const int64_t c0 = static_cast<int64_t>(pieces[3 * blockIdx.x + 2]) * tw;
  const int wlen = static_cast<int>((n_cols - c0) < tw ? (n_cols - c0) : tw);
  constexpr int PT = W / kXtGatherBlock;
  const int q0 = g0 >> 3, q1 = g1 >> 3;  // 8-entry groups
  const u32x4 *cv = reinterpret_cast<const u32x4 *>(col16);
  u32x4 w[U];
#ifdef LHPC_XT_PROBE_GVAL
  typedef T gv16 __attribute__((ext_vector_type(16 / sizeof(T))));
  constexpr int GVN = 8 * sizeof(T) / 16;  // 16-B vectors per 8 entries
  gv16 gv[U][GVN];
#endif
  auto load_w = [&](int q) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qq = q + u * kXtGatherBlock;
      w[u] = qq < q1 ? __builtin_nontemporal_load(cv + qq) : u32x4{0, 0, 0, 0};
#ifdef LHPC_XT_PROBE_GVAL
      const gv16 *vp = reinterpret_cast<const gv16 *>(vg + ((static_cast<int64_t>(qq) * 8) & vmask));
#pragma unroll
      for (int h = 0; h < GVN; ++h) gv[u][h] = __builtin_nontemporal_load(vp + h);
#endif
    }
  };
  load_w(q0 + tid);
  T tvv[PT];
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int j = i * kXtGatherBlock + tid;
    tvv[i] = j < wlen ? x[c0 + j] : T(0);
  }
#pragma unroll
  for (int i = 0; i < PT; ++i) xt[i * kXtGatherBlock + tid] = tvv[i];
  __syncthreads();
  typedef T tv16 __attribute__((ext_vector_type(16 / sizeof(T))));
  constexpr int VW = 16 / sizeof(T);
  if (pext) {
    const int delta = pext[2 * blockIdx.x], flags = pext[2 * blockIdx.x + 1];
    xg += delta;  // a multiple of 8: the 16-B store alignment holds
    if (tid < 2 && ((flags >> tid) & 1)) {
      const int gq = tid == 0 ? q0 - 1 : q1;  // the shared group before / at the end of the piece
      const u32x4 wq = cv[gq];
      T o[8];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        LHPC_DEVICE_CHECK((wq[h] & 0xFFFFu) < static_cast<uint32_t>(W) && (wq[h] >> 16) < static_cast<uint32_t>(W));
        o[2 * h] = xt[wq[h] & 0xFFFFu];
        o[2 * h + 1] = xt[wq[h] >> 16];
      }
#pragma unroll
      for (int h = 0; h < 8 / VW; ++h) {
        tv16 v;
#pragma unroll
        for (int k = 0; k < VW; ++k) v[k] = o[h * VW + k];
        *reinterpret_cast<tv16 *>(xg + static_cast<int64_t>(gq) * 8 + h * VW) = v;
      }
    }
  }
  for (int q = q0 + tid; q < q1; q += U * kXtGatherBlock) {
    if (q != q0 + tid) load_w(q);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qq = q + u * kXtGatherBlock;
      T o[8];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        LHPC_DEVICE_CHECK((w[u][h] & 0xFFFFu) < static_cast<uint32_t>(W) && (w[u][h] >> 16) < static_cast<uint32_t>(W));
        o[2 * h] = xt[w[u][h] & 0xFFFFu];
        o[2 * h + 1] = xt[w[u][h] >> 16];
      }
#ifdef LHPC_XT_PROBE_GVAL
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] *= gv[u][k / (16 / sizeof(T))][k % (16 / sizeof(T))];
#endif
      // a full 64-group block of the piece is stored wave-coalesced: the
      // plan permuted its col16 (xtile_gather_pos) so that the lane's 16-B
      // vector h lands at block + h·64·VW + VW·lane and every store
      // instruction writes 1 KB contiguous; a partial last block keeps the
      // lane's 8 entries contiguous
      const int qb = qq - lane;  // the wave's block (wave-uniform)
      T *blk = xg + static_cast<int64_t>(qb) * 8;
      if (qb + kWave <= q1) {
#pragma unroll
        for (int h = 0; h < 8 / VW; ++h) {
          tv16 v;
#pragma unroll
          for (int k = 0; k < VW; ++k) v[k] = o[h * VW + k];
#if defined(LHPC_XT_PROBE_GROUPED)
          // timing-only probe (wrong results): the store pattern of a tile-
          // grouped xg layout — groups of G tiles on one XCD (blocks with
          // equal b % 8, consecutive b / 8), every (tile, chunk) segment 9
          // 16-B units, stored at ((group·Cp + chunk)·G + tile in group)·9 + j
          {
            constexpr int G = LHPC_XT_PROBE_GROUPED, LQ = 9;
            const int bx = blockIdx.x % 8, bj = blockIdx.x / 8;
            const int64_t gi = (bj / G) * 8 + bx, tg = bj % G;
            const int64_t qv = static_cast<int64_t>(qb - q0) * 8 / VW + h * kWave + lane;  // 16-B unit in the piece
            const int64_t cp = static_cast<int64_t>(q1 - q0) * 8 / VW / LQ + 1;
            const int64_t units = static_cast<int64_t>(gridDim.x) * cp * LQ;  // ≈ the launch's share of xg
            const int64_t d = (((gi * cp + qv / LQ) * G + tg) * LQ + qv % LQ) % units;
            tv16 *a = reinterpret_cast<tv16 *>(xg) + d;
            if constexpr (NT) __builtin_nontemporal_store(v, a);
            else *a = v;
          }
#else
          tv16 *a = reinterpret_cast<tv16 *>(blk + h * kWave * VW + VW * lane);
          if constexpr (NT) __builtin_nontemporal_store(v, a);
          else *a = v;
#endif
        }
      } else if (qq < q1) {
#pragma unroll
        for (int h = 0; h < 8 / VW; ++h) {
          tv16 v;
#pragma unroll
          for (int k = 0; k < VW; ++k) v[k] = o[h * VW + k];
          tv16 *a = reinterpret_cast<tv16 *>(blk + 8 * lane + h * VW);
          if constexpr (NT) __builtin_nontemporal_store(v, a);
          else *a = v;
        }
      }
    }
  }
}

// reduce: one block per chunk c = C − 1 − ((b % 8)·Cx + b / 8), so each XCD
// walks a contiguous run of chunks and the xg lines two neighbouring chunks
// share stay in its L2; last chunks first, so the xg the gather wrote last
// (still in the Infinity Cache) is read first (C2 with cache-sized ranges:
// reduce 296 → 291 µs same box; C3 unchanged).  Both phases are branch-free
// and every load that does not depend on another is issued together (three
// round trips per chunk: the 16-B chunk descriptor {e0, e1, r0, r1} with the
// segment table; val run + row_ptr; xg (+ perm / iperm)):
//   scan     the chunk's S segment lengths are prefix-summed (with a count of
//            non-empty segments packed in the high half), giving each
//            non-empty segment its rank, base_ne[rank] = segment start −
//            flat offset, and a bit at its flat offset in sbm (M bits).
//   phase A  flat position f of the segment concatenation lies in the
//            non-empty segment of rank popcount(sbm bits ≤ f) − 1: a wave
//            prefix-scan of the sbm words gives each 64-position batch its
//            base rank, mbcnt gives the lane's; src = base_ne[rank] + f.
//            perm mode: xs[perm[src]] = xg[src] (CSR slot order); iperm mode:
//            xs[f] = xg[src] (flat order, fp32 by LDS-DMA).
//   phase B  thread t owns the run [RUN·t, RUN·t+RUN) (iperm mode: gathered
//            from xs through iperm[e0 + i]); a bitmap of row starts drives a
//            segmented scan (reset at a start, fma), whose running value
//            rounded to T is written back in place: a row that ends inside a
//            run leaves its value at its last position.  Rows crossing runs
//            are combined by a segmented scan over the threads, rows crossing
//            chunks leave fp64 pieces in `carry`, and the owned rows' y is
//            stored coalesced from their last positions.
#ifndef LHPC_XT_RBLK32
#define LHPC_XT_RBLK32 512
#endif
#ifndef LHPC_XT_RBLK64
#define LHPC_XT_RBLK64 1024
#endif
// reduce configurations: BLK threads, each owning one 64-B run of RUN =
// 64/sizeof(T) nonzeros (fp32 16, fp64 8); chunks of M = RUN·BLK nonzeros
// owning ≤ Rmax rows.  A 64-B run keeps LDS per wave at 4 KB for both types,
// so LDS never caps occupancy below 8 waves per SIMD.  fp32: BLK = 512 (C2
// reduce: 256 → 512 took 470 → 420 µs, 1024 was no faster).  fp64 with
// 16-nonzero runs held 8 KB per wave (73 KB per 512-thread block: 2 blocks,
// 16 waves per CU; C3 reduce 987 µs).
template <typename T> constexpr int xt_run() { return 64 / static_cast<int>(sizeof(T)); }
template <typename T, int BLK> struct XtRed {
  static constexpr int M = BLK * xt_run<T>(), Rmax = M / 8;
};
template <typename T> constexpr int xt_red_blk() { return sizeof(T) == 4 ? LHPC_XT_RBLK32 : LHPC_XT_RBLK64; }
// LDS slot of chunk position i (lhpc_plan.hpp xtile_slot): run t = i/RUN
// occupies 64 B at 64·t and its 16-B slot q is stored at q ^ xt_swz(t), so
// the 16 lanes of a ds_read_b128 group hit 16 distinct bank quads (4 runs per
// 256-B bank row, swizzled by the row's index mod 4)
__device__ __forceinline__ int xt_swz(int t) { return (t >> 2) & 3; }
template <typename T> __device__ __forceinline__ int xt_slot(int i) {
  constexpr int VW = 16 / sizeof(T), RUN = xt_run<T>();
  return (i & ~(RUN - 1)) | ((((i & (RUN - 1)) / VW) ^ xt_swz(i / RUN)) * VW) | (i & (VW - 1));
}

// Diagnostic build only (-DLHPC_XT_STAMPS, tools/xt_stamps.py): thread 0 of
// every reduce block records s_memrealtime at entry and exit and s_memtime at
// each phase boundary into g_xt_stamps[block][10]; never in a product build.
#ifdef LHPC_XT_STAMPS
__device__ uint64_t g_xt_stamps[1 << 22];
#define LHPC_XT_STAMP(i, real)                                                                  \
  if (threadIdx.x == 0)                                                                         \
    g_xt_stamps[static_cast<uint64_t>(blockIdx.x) * 10 + (i)] =                                 \
        (real) ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
#else
#define LHPC_XT_STAMP(i, real)
#endif

#ifndef LHPC_XT_XG_CPOL
// xg LDS-DMA cache policy.  With cache-sized ranges (C2, same box, two runs
// each): default 0 → reduce 292 µs; nt (2) 381 µs; sc0 (1) 292 µs; sc1 (16) 303 µs
#define LHPC_XT_XG_CPOL 0
#endif
#ifndef LHPC_XT_IP_WAVES
#define LHPC_XT_IP_WAVES 8  // iperm reduce: 8 waves/SIMD (fp32 66 → 64 VGPRs: C2 593 → 580 µs)
#endif
// the reduce keeps the chunk's row offsets in registers (k_xtile_reduce)
template <typename T> constexpr bool xt_rreg(int G) { return std::is_same<T, float>::value && G == 2; }

// AL (iperm only): aligned segments (lhpc_plan.hpp build_xtile unit > 1) —
// every segment starts on a 16-B boundary and spans whole 16-B units of VW
// positions, so phase A ranks units instead of positions (M/VW ≤ 64 batches
// of 64 units) and each lane moves one 16-B unit by LDS-DMA, fp64 included.
// PRE (iperm, no aligned segments; round 6): the plan holds each chunk's
// phase-A tables — the rank terms of its M/64 batches (bt, u32x4: start mask
// w >> 1 and the starts before the batch) and the bases of its non-empty
// segments (base_ne, S i32, ring positions) — and the reduce copies them
// into LDS by LDS-DMA in round trip 1 instead of the segment scan.
// seg = pbt (u32x4 per batch, as u32), seghi = pbne in that mode.
template <typename T, int G, int BLK, bool IP, bool AL, bool PRE = false>
__global__ __launch_bounds__(BLK, IP ? LHPC_XT_IP_WAVES : 1) void k_xtile_reduce(
    const int32_t *__restrict__ cdesc, const uint32_t *__restrict__ seg, const int32_t *__restrict__ seghi, int S,
    int64_t hc0, int64_t hrow0, int64_t c0, int64_t C,
    int64_t Cx, int total, const T *__restrict__ xg, const uint16_t *__restrict__ perm,
    const T *__restrict__ val, const int32_t *__restrict__ rp, T *__restrict__ y,
    double *__restrict__ carry, int y_add) {
  constexpr int RUN = xt_run<T>(), M = XtRed<T, BLK>::M, RMAX = XtRed<T, BLK>::Rmax;
  constexpr int RPT = (RMAX + 1 + BLK - 1) / BLK;  // row_ptr loads per thread
  constexpr int NB = M / BLK;                      // 64-position batches per wave (= RUN)
  static_assert((NB == 16 || NB == 8) && M <= 256 * kWave && M >= 4096,
                "8/16 batches per wave; ≤ 256 batches per chunk; sbm ≥ 128 words");
  typedef T tvec __attribute__((ext_vector_type(16 / sizeof(T)), aligned(sizeof(T))));
  constexpr int VW = 16 / sizeof(T), NV = RUN / VW;
  static_assert(!AL || IP, "aligned segments need the iperm reduce");
  constexpr int NBU = NB / VW;  // AL: 64-unit batches per wave
  static_assert(!AL || NBU * (BLK / kWave) <= kWave, "AL: a chunk's unit batches fit one wave's lanes");
  // dynamic LDS (xtile_lds_bytes): xs[M + VW] T (slot M is the sentinel's
  // spare), bt[BLK/64][NB] u32x4, ws[BLK/64] f64, wsf[BLK/64] i32, bm[M/32]
  // u32, sbm[M/32] u32, rfirst[RPT][BLK/64] u16 (padded to 4 B), rlast i32,
  // base_ne[S] i32, wsum[16] i32 (one per wave: fp64 blocks have 16).  RREG (fp32 G = 2, 476–1024 tiles): the
  // chunk's local row offsets stay in the threads' registers (rt[q] = row
  // q·BLK + tid) and the y store takes row j+1's from lane + 1, or from
  // rfirst for a wave's last lane — 56 B of LDS instead of rpl[RMAX+1] u16
  // (2 KB), so the fp32 reduce keeps 4 blocks per CU up to ≈ 970 tiles
  // instead of ≈ 470 (same box: n = 30M +1.1%, 80M +3.3%).  Only fp32 G = 2
  // gains: G = 1 plans (C2) keep rpl in LDS (the register form cost C2
  // 0.8%), and past 1024 tiles base_ne alone exceeds the 4-block budget.
  constexpr bool RREG = xt_rreg<T>(G);
  extern __shared__ __align__(16) unsigned char smem[];
  T *xs = reinterpret_cast<T *>(smem);
  u32x4 *bt0 = reinterpret_cast<u32x4 *>(xs + M + VW);
  double *ws = reinterpret_cast<double *>(bt0 + (BLK / kWave) * NB);  // per-wave segmented-scan totals
  int *wsf = reinterpret_cast<int *>(ws + BLK / kWave);
  uint32_t *bm = reinterpret_cast<uint32_t *>(wsf + BLK / kWave);
  uint32_t *sbm = bm + M / 32;
  constexpr int NW = BLK / kWave;
  uint16_t *rpl = reinterpret_cast<uint16_t *>(sbm + M / 32);  // !RREG: rpl[RMAX + 1]
  uint16_t *rfirst = rpl;                                       // RREG: rfirst[RPT][NW]
  int32_t *rlast = reinterpret_cast<int32_t *>(rfirst + ((RPT * NW + 1) & ~1));
  int32_t *base_ne = RREG ? rlast + 1 : reinterpret_cast<int32_t *>(rpl + ((RMAX + 2) & ~1));
  int32_t *wsum = base_ne + S;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int i0 = tid * RUN;
  const int64_t c = C - 1 - (static_cast<int64_t>(blockIdx.x % 8) * Cx + blockIdx.x / 8);  // chunk range [c0, C)
  if (c < c0) return;  // block-uniform
  LHPC_XT_STAMP(0, 1)
  LHPC_XT_STAMP(1, 0)
  // ---- round trip 1: the chunk descriptor and the segment table (both
  //      addressed by c alone), then — without waiting for them — round
  //      trip 2 (val run and row_ptr, addressed by the descriptor).  The
  //      segment scan and phase A need only the table, so phase A's xg loads
  //      go out while val and row_ptr are still in flight.
  static_assert(!PRE || (IP && !AL), "PRE: the iperm reduce without aligned segments");
  int sa[G], sb[G];
  if constexpr (PRE) {
#if defined(__HIP_DEVICE_COMPILE__)
    // the chunk's phase-A tables into LDS: bt (M/64 u32x4 = M/16 dwords,
    // 64 per wave instruction) and base_ne (S dwords, padded to 64 in LDS)
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t *>(seg + c * (M / 16)), 0, (M / 16) * 4, 0x00020000);
    for (int k = wv; k < M / 16 / kWave; k += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void *)(reinterpret_cast<uint32_t *>(bt0) + k * kWave),
                                               4, (k * kWave + lane) * 4, 0, 0, 0);
    const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int32_t *>(seghi + c * S), 0, S * 4, 0x00020000);
    for (int k = wv; k * kWave < S; k += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rn, (__attribute__((address_space(3))) void *)(base_ne + k * kWave), 4,
                                               (k * kWave + lane) * 4, 0, 0, 0);
#endif
    (void)sa;
    (void)sb;
  } else {
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int sI = tid * G + q;
      const int sc = sI < S ? sI : S - 1;
      // segment table (lhpc_plan.hpp xtile_segment_table): start = hi + lo, end = start + len
      const uint32_t w = seg[c * S + sc];
      // hi row: ⌊c / kXtSegHi⌋, or per range in ring plans (hrow0 + ⌊(c − hc0) / kXtSegHi⌋)
      sa[q] = seghi[(hrow0 + (c - hc0) / kXtSegHi) * S + sc] + static_cast<int>(w & 0xFFFFu);
      sb[q] = sa[q] + static_cast<int>(w >> 16);
    }
  }
  const u32x4 d = *reinterpret_cast<const u32x4 *>(cdesc + 8 * c);
  const u32x4 d2 = *reinterpret_cast<const u32x4 *>(cdesc + 8 * c + 4);
  const int e0 = static_cast<int>(d[0]), m = static_cast<int>(d[1]) - e0;
  const int r0 = static_cast<int>(d[2]), R = static_cast<int>(d[3]) - r0;
  // val and iperm are stored wave-transposed (lhpc_plan.hpp xtile_wave_pos):
  // in the chunk's wave region w (REG = 64·RUN positions at vbase + w·REG),
  // 16-B vector q of lane l holds that lane's run elements [q·VW, q·VW + VW),
  // so each load instruction reads 1 KB contiguous (per-lane runs touched
  // every 128-B line with 2 lanes per instruction: 4× the L2 requests for
  // val).  A wave whose region starts past m reads region 0 (masked below).
  constexpr int REG = kWave * RUN;
  const int64_t vreg = static_cast<int64_t>(static_cast<int>(d2[0])) + (wv * REG < m ? wv : 0) * REG;
  tvec vv[NV];
  {
    const tvec *vp = reinterpret_cast<const tvec *>(val + vreg) + lane;
#pragma unroll
#if defined(LHPC_XT_PROBE_VI) || defined(LHPC_XT_PROBE_NOVAL)  // timing-only probe: no val (/ iperm) loads
    for (int q = 0; q < NV; ++q) vv[q] = tvec{};
    (void)vp;
#else
    for (int q = 0; q < NV; ++q) vv[q] = __builtin_nontemporal_load(vp + q * kWave);
#endif
  }
  constexpr int NIP = IP ? RUN * 2 / 16 : 1;  // 16-B iperm vectors per run
  u32x4 ipv[NIP];
  // iperm: loaded once phase A's xg loads are issued, so it is not live
  // during the rank math; padding entries are 0 (a valid LDS slot)
  auto load_ipv = [&]() {
    const u32x4 *ip = reinterpret_cast<const u32x4 *>(perm + vreg) + lane;
#pragma unroll
#if defined(LHPC_XT_PROBE_VI)
    for (int q = 0; q < NIP; ++q) ipv[q] = u32x4{0, 0, 0, 0};
    (void)ip;
#else
    for (int q = 0; q < NIP; ++q) ipv[q] = __builtin_nontemporal_load(ip + q * kWave);
#endif
  };
  int rv[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int j = q * BLK + tid;
    rv[q] = rp[r0 + (j <= R ? j : R)];
  }
  // ---- scan: segment ranks / bases and the segment-start bitmap (PRE:
  //      the plan's tables, once their LDS-DMA has landed)
  if (tid < M / 32) {
    bm[tid] = 0u;
    sbm[tid] = 0u;
  }
  if constexpr (PRE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
  int lsum = 0;  // (length | non-empty count << 16) of this thread's segments
#pragma unroll
  for (int q = 0; q < G; ++q) {
    if (tid * G + q >= S) sb[q] = sa[q];
    lsum += (sb[q] - sa[q]) + (sb[q] > sa[q] ? 0x10000 : 0);
  }
  const int inc = wave_incl_scan(lsum);
  if (lane == kWave - 1) wsum[wv] = inc;
  __syncthreads();
  LHPC_XT_STAMP(2, 0)
  {
    int run = inc - lsum;
    for (int w = 0; w < wv; ++w) run += wsum[w];
    int off = run & 0xFFFF, rank = run >> 16;
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int len = sb[q] - sa[q];
      if (len > 0) {
        base_ne[rank] = sa[q] - off;
        const int ub = AL ? off / VW : off;  // AL: the bitmap marks start units
        LHPC_DEVICE_CHECK(!AL || (off % VW == 0 && sa[q] % VW == 0));
        atomicOr(sbm + (ub >> 5), 1u << (ub & 31));
        ++rank;
      }
      off += len;
    }
  }
  __syncthreads();
  }  // !PRE
  LHPC_XT_STAMP(3, 0)

  // ---- phase A: src = base_ne[rank] + f, xg loads (round trip 3);
  //      positions past m load the sentinel entry `total` (perm: spare slot M)
  int src[NB];
  if constexpr (AL) {
    // unit u of batch j covers flat positions VW·((wv·NBU + j)·64 + lane) …;
    // lane q holds unit batch q's bitmap word (≤ 64 batches: one pass)
    const uint64_t wl = static_cast<uint64_t>(sbm[2 * lane]) | (static_cast<uint64_t>(sbm[2 * lane + 1]) << 32);
    const int cnt = __popcll(wl);
    const int incl = wave_incl_scan(cnt);
    u32x4 *bt = bt0 + wv * NB;
    if (lane / NBU == wv) {
      const uint64_t w1 = wl >> 1;
      bt[lane & (NBU - 1)] = u32x4{static_cast<uint32_t>(w1), static_cast<uint32_t>(w1 >> 32),
                                   static_cast<uint32_t>(incl - cnt - 1 + static_cast<int>(wl & 1u)), 0u};
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < NBU; ++u) {
      const u32x4 t = bt[u];
      const int rk = __builtin_amdgcn_mbcnt_hi(t[1], __builtin_amdgcn_mbcnt_lo(t[0], t[2]));
      src[u] = base_ne[rk] + ((wv * NBU + u) * kWave + lane) * VW;  // a multiple of VW: 16-B aligned
    }
  } else {
    // lane q holds batch q's word; the wave-uniform rank terms (w >> 1,
    // base) go to an LDS triple that the owning wave reads back as a
    // broadcast:  rank = starts before the batch − 1 + (w & 1) + mbcnt(w >> 1)
    // (lanes hold batch words q and q + 64 … when M > 4096); wave w owns
    // batches [NB·w, NB·w + NB)
    u32x4 *bt = bt0 + wv * NB;
    if constexpr (!PRE) {
      const int grp = (wv * NB) >> 6;  // this wave's batches lie in 64-batch group grp
      uint64_t wl = 0;
      int cnt = 0, incl = 0, below = 0;
      for (int g2 = 0; g2 <= grp; ++g2) {  // wave-uniform
        wl = static_cast<uint64_t>(sbm[128 * g2 + 2 * lane]) | (static_cast<uint64_t>(sbm[128 * g2 + 2 * lane + 1]) << 32);
        cnt = __popcll(wl);
        incl = wave_incl_scan(cnt) + below;  // starts in batches ≤ 64·g2 + lane
        below = __builtin_amdgcn_readlane(incl, kWave - 1);
      }
      if (lane / NB == wv % (kWave / NB)) {  // lanes holding this wave's batches
        const uint64_t w1 = wl >> 1;
        bt[lane & (NB - 1)] = u32x4{static_cast<uint32_t>(w1), static_cast<uint32_t>(w1 >> 32),
                                    static_cast<uint32_t>(incl - cnt - 1 + static_cast<int>(wl & 1u)), 0u};
      }
      __builtin_amdgcn_wave_barrier();  // LDS is in order within a wave: no block barrier needed
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const u32x4 t = bt[u];  // uniform address: broadcast
      const int rk = __builtin_amdgcn_mbcnt_hi(t[1], __builtin_amdgcn_mbcnt_lo(t[0], t[2]));
      const int f = (wv * NB + u) * kWave + lane;
      const int sv = base_ne[rk] + f;  // m > 0 ⇒ 0 ≤ rk < S; m = 0: base_ne[−1] (in LDS), unused
      if constexpr (IP)
        src[u] = sv;  // past m: out-of-chunk or out-of-range data into never-read slots
      else
        src[u] = f < m ? sv : total;
      LHPC_DEVICE_CHECK(IP || (src[u] >= 0 && src[u] <= total));
    }
  }
  // plain loads: the segment lines a neighbouring chunk shares must stay in
  // L2 (non-temporal xg/perm loads: 433 → 555 µs)
  if constexpr (IP) {
    // buffer loads with 32-bit offsets (the plan keeps the xg stream < 2 GiB
    // in this mode): a position past m loads whatever follows its segment, or
    // 0 past the stream's end (out of range) — no select and no 64-bit
    // address per load; those slots are never read (padded positions read
    // the zero slot M).  Default cache policy: the lines two neighbouring
    // chunks' segments share must stay in L2 (nt / sc0+nt / sc1+nt: C2
    // 524 → 554 µs; sc0 523, sc1 527, sc0+sc1 527 µs; one tile with no shared
    // lines: nt 354 → 331 µs, nt + 16-B LDS-DMA 306 µs — DESIGN.md §4)
    const __amdgpu_buffer_rsrc_t xr_rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T *>(xg), 0, (total + 2) * static_cast<int>(sizeof(T)), 0x00020000);
    if constexpr (AL) {
      // one 16-B unit per lane, straight into its flat slots (64 units = 1 KB
      // of LDS per instruction); a unit past the chunk loads what follows its
      // segment (or 0 past the stream) into slots nothing reads.  Device pass
      // only: the host pass's semantic check rejects the 16-B size (a gfx950
      // feature) without a diagnostic and then drops the kernel's host stub
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
      for (int u = 0; u < NBU; ++u)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xr_rs, (__attribute__((address_space(3))) void *)(xs + (wv * NBU + u) * kWave * VW), 16,
            src[u] * static_cast<int>(sizeof(T)), 0, 0, LHPC_XT_XG_CPOL);
#endif
      load_ipv();
    } else if constexpr (sizeof(T) == 4) {
#if defined(LHPC_XT_PROBE_XG)
      // timing-only probe (wrong results): 1 = the chunk's xg as one aligned
      // contiguous run, 16-B LDS-DMA per lane; 2 = the same, non-temporal;
      // 3 = no xg loads; 4 = one contiguous run, 4-B LDS-DMA per lane
      if constexpr (LHPC_XT_PROBE_XG == 1 || LHPC_XT_PROBE_XG == 2) {
#pragma unroll
        for (int u = 0; u < NB / 4; ++u)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              xr_rs, (__attribute__((address_space(3))) void *)(xs + (wv * NB + 4 * u) * kWave), 16,
              static_cast<int>((c * M + (wv * NB + 4 * u) * kWave + 4 * lane) * 4), 0, 0,
              LHPC_XT_PROBE_XG == 2 ? 2 : 0);
      } else if constexpr (LHPC_XT_PROBE_XG == 4) {
#pragma unroll
        for (int u = 0; u < NB; ++u)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              xr_rs, (__attribute__((address_space(3))) void *)(xs + (wv * NB + u) * kWave), 4,
              static_cast<int>((c * M + (wv * NB + u) * kWave + lane) * 4), 0, 0, 0);
      }
      (void)src;
#else
      // LDS-DMA: each lane's xg element lands at the batch's base + 4·lane
      // (exactly the flat order), no VGPR destination
#pragma unroll
      for (int u = 0; u < NB; ++u)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xr_rs, (__attribute__((address_space(3))) void *)(xs + (wv * NB + u) * kWave), 4,
            src[u] * static_cast<int>(sizeof(T)), 0, 0, LHPC_XT_XG_CPOL);
#endif
      load_ipv();
    } else {
#if defined(LHPC_XT_PROBE_XG)
      // timing-only probes, fp64: 1 = contiguous 16-B loads per lane (two
      // positions each) + ds_write_b128; 3 = none; 4 = contiguous 8-B loads
      if constexpr (LHPC_XT_PROBE_XG == 1 || LHPC_XT_PROBE_XG == 2) {
        typedef double d2 __attribute__((ext_vector_type(2)));
        d2 xv[NB / 2];
#pragma unroll
        for (int u = 0; u < NB / 2; ++u)
          xv[u] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(
                                             xr_rs, static_cast<int>((c * M + (wv * NB + 2 * u) * kWave + 2 * lane) * 8), 0,
                                             LHPC_XT_PROBE_XG == 2 ? 2 : 0));
#pragma unroll
        for (int u = 0; u < NB / 2; ++u) *reinterpret_cast<d2 *>(xs + (wv * NB + 2 * u) * kWave + 2 * lane) = xv[u];
      } else if constexpr (LHPC_XT_PROBE_XG == 4) {
        T xv[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u)
          xv[u] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(
                                            xr_rs, static_cast<int>((c * M + (wv * NB + u) * kWave + lane) * 8), 0, 0));
#pragma unroll
        for (int u = 0; u < NB; ++u) xs[(wv * NB + u) * kWave + lane] = xv[u];
      }
      (void)src;
#else
      // (a 4-B LDS-DMA form, two instructions per 64 positions, was 2%
      // slower: DESIGN.md §4.1 round 6)
      T xv[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u)
        xv[u] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(xr_rs, src[u] * 8, 0, 0));
#pragma unroll
      for (int u = 0; u < NB; ++u) xs[(wv * NB + u) * kWave + lane] = xv[u];
#endif
      load_ipv();
    }
  } else {
    T xv[NB];
    uint16_t pv[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      xv[u] = xg[src[u]];
      pv[u] = perm[src[u]];  // LDS slot xt_slot(position); the sentinel's: M
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) xs[pv[u]] = xv[u];
  }
  LHPC_XT_STAMP(4, 0)
  // row_ptr (round trip 2) → local row offsets (registers; a wave's first in
  // rfirst, row R's in rlast) and the row-start bitmap
  int rt[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int j = q * BLK + tid;
    rv[q] -= e0;
    rt[q] = rv[q] <= m ? rv[q] : m + 1;  // > m: continues (rows past R repeat row R's)
    if constexpr (RREG) {
      if (lane == 0) rfirst[q * NW + wv] = static_cast<uint16_t>(rt[q]);
      if (j == R) *rlast = rt[q];
    } else {
      if (j <= R) rpl[j] = static_cast<uint16_t>(rt[q]);
    }
    if (j < R && rv[q] < m) atomicOr(bm + (rv[q] >> 5), 1u << (rv[q] & 31));  // empty rows share a bit
  }
  const int n = m - i0 < RUN ? (m - i0 > 0 ? m - i0 : 0) : RUN;  // valid entries in the run
  if (n < RUN) {  // the chunk's last run (and runs past m): val and x past m → 0 · 0
    if constexpr (!IP)
      for (int j = n; j < RUN; ++j) xs[xt_slot<T>(i0 + j)] = T(0);
#pragma unroll
    for (int j = 0; j < RUN; ++j) vv[j / VW][j % VW] = j < n ? vv[j / VW][j % VW] : T(0);
  }
  if constexpr (IP)
    if (tid == 0) xs[M] = T(0);  // the zero slot that iperm padding points at
  // the LDS-DMA of phase A is counted by vmcnt, which the barrier does not
  // wait for: drain it before any wave reads another wave's flat slots
  if constexpr (IP && (sizeof(T) == 4 || AL)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  LHPC_XT_STAMP(5, 0)

  // ---- phase B: branch-free segmented scan of the thread's run.  The fp32
  //      product is exact in fp64, so the fma equals the add of the product.
  const uint32_t mask = (bm[i0 >> 5] >> (i0 & 31)) & ((1u << RUN) - 1u);
  const int hl = mask ? __builtin_ctz(mask) : RUN;  // head length (entries before the first start)
  const int hend = (hl < n ? hl : n) - 1;                // last head position (−1: none)
  // the run is NV 16-B slots at RUN·tid, slot q stored at q ^ xt_swz (conflict-free ds_read_b128)
  typedef T lvec __attribute__((ext_vector_type(VW)));
  lvec *xr = reinterpret_cast<lvec *>(xs + i0);
  const int swz = xt_swz(tid);
  lvec xq[NV];
  if constexpr (IP) {
    // gather the run's x from the flat array, then (after every thread has
    // read) the running sums below go back in the CSR (xt_slot) layout;
    // unconditional reads, so all RUN ds_reads issue before the first wait.
    // A padded position's iperm is the zero slot M, so x past m is already
    // 0 (a run wholly past m reads another region's iperm: n = 0, unused)
#pragma unroll
    for (int j = 0; j < RUN; ++j) {
      const uint32_t w = ipv[j / 8][(j % 8) / 2];
      LHPC_DEVICE_CHECK(((j & 1) ? (w >> 16) : (w & 0xFFFFu)) < static_cast<uint32_t>(M + VW));
      xq[j / VW][j % VW] = xs[static_cast<int>((j & 1) ? (w >> 16) : (w & 0xFFFFu))];
    }
    __syncthreads();
  } else {
#pragma unroll
    for (int q = 0; q < NV; ++q) xq[q] = xr[q ^ swz];
  }
  double acc = 0.0, hsave = 0.0;
#pragma unroll
  for (int j = 0; j < RUN; ++j) {
    acc = ((mask >> j) & 1u) ? 0.0 : acc;
    acc = __builtin_fma(static_cast<double>(vv[j / VW][j % VW]), static_cast<double>(xq[j / VW][j % VW]), acc);
    hsave = j == hend ? acc : hsave;
    xq[j / VW][j % VW] = static_cast<T>(acc);  // in place; slots past m are never read
  }
#pragma unroll
  for (int q = 0; q < NV; ++q) xr[q ^ swz] = xq[q];
  const bool has_head = n > 0 && !(mask & 1u);
  const bool cont = (RREG ? *rlast : static_cast<int>(rpl[R])) > m;  // the row active at m−1 runs past the chunk
  // ---- rows that cross runs: segmented scan over threads (run order) of
  //      x(t) = tail piece if run t holds a row start, else its whole-run sum;
  //      the row open when run t begins is the exclusive value S(t−1)
  bool fl = n > 0 && mask != 0u;
  double sv = wave_seg_scan(fl ? acc : hsave, fl);
  if (lane == kWave - 1) {
    ws[wv] = sv;
    wsf[wv] = fl ? 1 : 0;
  }
  __syncthreads();
  double cw = 0.0;  // segmented carry of the waves before this one
  int gw = 0;
  for (int w = 0; w < wv; ++w) {
    cw = wsf[w] ? ws[w] : cw + ws[w];
    gw |= wsf[w];
  }
  LHPC_XT_STAMP(6, 0)
  if (!fl) sv = cw + sv;
  const int fin_incl = (fl ? 1 : 0) | gw;
  constexpr int kShr1 = 0x138;  // DPP wave_shr:1 (lane l ← lane l−1; lane 0 keeps `old`)
  const double oin = dpp_f64_old<kShr1>(cw, sv);                                 // S(t−1)
  const int fin = __builtin_amdgcn_update_dpp(gw, fin_incl, kShr1, 0xF, 0xF, false);  // starts before run t
  const int tlast = m > 0 ? (m - 1) / RUN : -1;
  if (tid == 0 && !(m > 0 && (RREG ? rt[0] : static_cast<int>(rpl[0])) > 0)) carry[2 * c] = 0.0;  // no head piece
  if (has_head) {
    const int i1 = i0 + n;
    const bool end_i1 = i1 < m ? ((bm[i1 >> 5] >> (i1 & 31)) & 1u) != 0 : !cont;
    const bool ends = hl < n || end_i1;
    if (ends || tid == tlast) {
      const double sum = oin + hsave;
      if (!fin) {
        carry[2 * c] = sum;  // this chunk's piece of the previous chunk's row
      } else if (ends) {
        xs[xt_slot<T>(i0 + hend)] = static_cast<T>(sum);
      } else {
        carry[2 * c + 1] = sum;  // row continues into the next chunk
      }
    }
  }
  if (tid == tlast && mask && cont) carry[2 * c + 1] = acc;  // own tail row continues
  __syncthreads();
  LHPC_XT_STAMP(7, 0)
  // coalesced y store of the owned rows from their last positions (a row
  // continuing past the chunk is stored by k_xtile_fixup, later on the stream)
  // (y_add: a column block after the first adds its sums; empty rows keep y)
  if constexpr (RREG) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int j = q * BLK + tid;
      // row j + 1's offset: lane + 1's register (every lane shuffles), the
      // next wave's first (rfirst) for a wave's last lane; j < R keeps q + 1 < RPT
      int a1 = __shfl_down(rt[q], 1, kWave);
      if (lane == kWave - 1) a1 = wv + 1 < NW ? rfirst[q * NW + wv + 1] : (q + 1 < RPT ? rfirst[(q + 1) * NW] : 0);
      if (j < R) {
        const int a0 = rt[q];
        if (a1 == a0) {
          if (!y_add) y[r0 + j] = T(0);
        } else if (a1 <= m) {
          const T v = xs[xt_slot<T>(a1 - 1)];
          y[r0 + j] = y_add ? static_cast<T>(static_cast<double>(y[r0 + j]) + static_cast<double>(v)) : v;
        }
      }
    }
  } else {
    for (int j = tid; j < R; j += BLK) {
      const int a0 = rpl[j], a1 = rpl[j + 1];
      if (a1 == a0) {
        if (!y_add) y[r0 + j] = T(0);
      } else if (a1 <= m) {
        const T v = xs[xt_slot<T>(a1 - 1)];
        y[r0 + j] = y_add ? static_cast<T>(static_cast<double>(y[r0 + j]) + static_cast<double>(v)) : v;
      }
    }
  }
  LHPC_XT_STAMP(8, 0)
  LHPC_XT_STAMP(9, 1)
}

// rows cut by a chunk end: y[row] = tail piece + head pieces, chunk order
template <typename T>
__global__ __launch_bounds__(kXtFixBlock) void k_xtile_fixup(
    const int32_t *__restrict__ cont, int64_t n_cont, const int32_t *__restrict__ cr, int64_t C,
    const double *__restrict__ carry, T *__restrict__ y, int acc) {  // C: end of the chunk range (rows never cross it)
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kXtFixBlock + threadIdx.x;
  if (i >= n_cont) return;
  const int64_t c = cont[i];
  double s = carry[2 * c + 1];
  for (int64_t d = c + 1; d < C; ++d) {
    s += carry[2 * d];
    if (cr[d + 1] > cr[d]) break;
  }
  T *yr = y + (cr[c + 1] - 1);
  *yr = acc ? static_cast<T>(static_cast<double>(*yr) + s) : static_cast<T>(s);
}

// ------------------------------------------------------------ launchers
// segment-table entries per reduce thread: G = ⌈S / BLK⌉ rounded up to a
// power of two.  build_xtile caps S at kXtMaxTiles = 4096, so G ≤ 8 for fp32
// (BLK 512) and ≤ 4 for fp64 (BLK 1024); only those are instantiated (a G = 16
// form spilled and could never be selected)
template <typename T> constexpr int xt_gmax() { return 4096 / xt_red_blk<T>(); }
template <typename T>
size_t xtile_lds_bytes_g(int S, int g, bool pre = false) {
  constexpr int BLK = xt_red_blk<T>(), M = XtRed<T, BLK>::M, RMAX = XtRed<T, BLK>::Rmax, W = BLK / kWave;
  constexpr int RPT = (RMAX + 1 + BLK - 1) / BLK;
  const size_t rows = xt_rreg<T>(g) ? ((RPT * W + 1) & ~1) * sizeof(uint16_t) + sizeof(int32_t)  // rfirst, rlast
                                    : ((RMAX + 2) & ~1) * sizeof(uint16_t);                     // rpl
  return static_cast<size_t>(M + 16 / sizeof(T)) * sizeof(T) + W * xt_run<T>() * 16 + W * (sizeof(double) + 4) +
         2 * M / 32 * sizeof(uint32_t) + rows + sizeof(int32_t) * (static_cast<size_t>(S) + 16) +  // base_ne, wsum[BLK/64 ≤ 16]
         (pre ? 256 : 0);  // PRE: base_ne's LDS-DMA writes whole 64-entry rows
}
// a G = 1 plan whose rpl pushes the reduce past 4 blocks per CU (160 KB / 4
// of LDS; fp32 S ≈ 476–512) takes the G = 2 form, whose row offsets live in
// registers, when that one fits
constexpr size_t kXtLds4 = 160 * 1024 / 4;
template <typename T>
int xtile_g(int S) {
  const int g = (S + xt_red_blk<T>() - 1) / xt_red_blk<T>();
  if (g <= 1)
    return xt_rreg<T>(2) && xtile_lds_bytes_g<T>(S, 1) > kXtLds4 && xtile_lds_bytes_g<T>(S, 2) <= kXtLds4 ? 2 : 1;
  return g <= 2 ? 2 : g <= 4 ? 4 : 8;
}
template <typename T>
size_t xtile_lds_bytes(int S) {
  return xtile_lds_bytes_g<T>(S, xtile_g<T>(S));
}

template <typename T, int G, bool IP, bool AL, bool PRE = false>
const void *xtile_reduce_fn() {
  if constexpr (G > xt_gmax<T>() || (AL && !IP) || (AL && G > 4) || (PRE && (!IP || AL)))  // AL at G = 8 spilled
    return nullptr;
  else
    return reinterpret_cast<const void *>(k_xtile_reduce<T, G, xt_red_blk<T>(), IP, AL, PRE>);
}
template <typename T, bool IP, bool AL, bool PRE = false>
const void *xtile_reduce_fn(int g) {
  return g == 1 ? xtile_reduce_fn<T, 1, IP, AL, PRE>() : g == 2 ? xtile_reduce_fn<T, 2, IP, AL, PRE>()
         : g == 4 ? xtile_reduce_fn<T, 4, IP, AL, PRE>() : xtile_reduce_fn<T, 8, IP, AL, PRE>();
}
// ip: iperm reduce; al: aligned segments (iperm only, else nullptr); pre:
// the plan's phase-A tables instead of the segment scan (iperm, not aligned)
template <typename T>
const void *xtile_reduce_fn(int g, bool ip, bool al, bool pre = false) {
  if (pre) return ip && !al && g == 1 ? xtile_reduce_fn<T, 1, true, false, true>() : nullptr;  // G = 2 spilled
  if (al) return ip ? xtile_reduce_fn<T, true, true>(g) : nullptr;
  return ip ? xtile_reduce_fn<T, true, false>(g) : xtile_reduce_fn<T, false, false>(g);
}

template <typename T, int U, bool NT = false>
void gather_u(const lhpc_spmv_plan *p, const int32_t *pieces, const void *x, int64_t q0, int64_t q1, hipStream_t s,
              const int32_t *pext) {
#ifdef LHPC_XT_PROBE_GVAL
  int64_t vmask = 1;
  while (vmask * 2 <= p->nnz) vmask *= 2;
  vmask = (vmask - 1) & ~int64_t{7};
  if constexpr (U > LHPC_XT_PROBE_GVAL) {
    gather_u<T, LHPC_XT_PROBE_GVAL, NT>(p, pieces, x, q0, q1, s, pext);
    return;
  } else
    hipLaunchKernelGGL((k_xtile_gather<T, U, NT>), dim3(static_cast<unsigned>(q1 - q0)), dim3(kXtGatherBlock), 0, s,
                       pieces + 3 * q0, p->d_col16, static_cast<const T *>(x), p->n_cols,
                       static_cast<int>(p->xs_width), static_cast<T *>(p->d_xg), pext ? pext + 2 * q0 : nullptr,
                       static_cast<const T *>(p->d_val), vmask);
#else
  hipLaunchKernelGGL((k_xtile_gather<T, U, NT>), dim3(static_cast<unsigned>(q1 - q0)), dim3(kXtGatherBlock), 0, s,
                     pieces + 3 * q0, p->d_col16, static_cast<const T *>(x), p->n_cols,
                     static_cast<int>(p->xs_width), static_cast<T *>(p->d_xg), pext ? pext + 2 * q0 : nullptr);
#endif
}

// gather pieces [q0, q1) (default: all) of `pieces` (default: the plan's)
template <typename T>
int launch_gather(const lhpc_spmv_plan *p, const void *x, hipStream_t s, int64_t q0 = 0, int64_t q1 = -1,
                  const int32_t *pieces = nullptr) {
  if (q1 < 0) q1 = p->xt_pieces;
  if (q1 <= q0) return LHPC_OK;
  // the ring's per-piece deltas belong to the plan's own pieces
  const int32_t *pext = !pieces && p->xt_ring ? p->d_pext : nullptr;
  if (!pieces) pieces = p->d_pieces;
  if (p->xt_nt) {
    gather_u<T, 8, true>(p, pieces, x, q0, q1, s, pext);
    return check_launch(s);
  }
  switch (p->xt_u) {
    case 2: gather_u<T, 2>(p, pieces, x, q0, q1, s, pext); break;
    case 4: gather_u<T, 4>(p, pieces, x, q0, q1, s, pext); break;
    case 16:  // fp64 at 16 steps needs > 128 VGPRs (it spilled 22): capped at 8
      if constexpr (sizeof(T) == 8) gather_u<T, 8>(p, pieces, x, q0, q1, s, pext);
      else gather_u<T, 16>(p, pieces, x, q0, q1, s, pext);
      break;
    default: gather_u<T, 8>(p, pieces, x, q0, q1, s, pext); break;
  }
  return check_launch(s);
}

// reduce of chunks [c0, c1) into y (rows at their plan index), then the fix-up
// of the rows cut inside the range: cont entries [n0, n1)
// ring: range k of a ring plan (ring-sized xg, range k's hi rows); −1: the
// plan's whole stream
template <typename T>
int launch_reduce(const lhpc_spmv_plan *p, int64_t c0, int64_t c1, int64_t n0, int64_t n1, T *y,
                  hipStream_t s, int ring = -1) {
  if (c1 > c0) {
    const int64_t Cx = (c1 - c0 + 7) / 8;
    const dim3 rg(static_cast<unsigned>(8 * Cx)), rb(xt_red_blk<T>());
    const void *fn = xtile_reduce_fn<T>(xtile_g<T>(p->S), p->xt_p == 3, p->xt_al != 0, p->xt_pre != 0);
    const int32_t *cd = p->d_cdesc, *sh = p->d_seghi, *rp = static_cast<const int32_t *>(p->d_row_ptr);
    const uint32_t *so = p->d_seg;
    int S = p->S, total = static_cast<int>(ring >= 0 ? p->xt_ring_len : p->xt_total);
    int64_t hc0 = ring >= 0 ? c0 : 0, hrow0 = ring >= 0 ? p->xt_hrow[static_cast<size_t>(ring)] : 0;
    const T *xg = static_cast<const T *>(p->d_xg), *val = static_cast<const T *>(p->d_val);
    const uint16_t *perm = p->d_perm;
    double *carry = p->d_carry;
    int acc = p->xt_acc;
    void *args[] = {&cd, &so, &sh, &S, &hc0, &hrow0, &c0, &c1, const_cast<int64_t *>(&Cx), &total, &xg, &perm, &val,
                    &rp, &y, &carry, &acc};
    LHPC_HIP_TRY(hipLaunchKernel(fn, rg, rb, args, p->xt_lds, s));
    LHPC_TRY(check_launch(s));
  }
  if (n1 > n0) {
    hipLaunchKernelGGL((k_xtile_fixup<T>), dim3(static_cast<unsigned>((n1 - n0 + kXtFixBlock - 1) / kXtFixBlock)),
                       dim3(kXtFixBlock), 0, s, p->d_cont + n0, n1 - n0, p->d_cr, c1, p->d_carry, y, p->xt_acc);
    LHPC_TRY(check_launch(s));
  }
  return LHPC_OK;
}


// ---------------------------------------------- device-side layout build
// The O(nnz) passes of the XTILE layout from device-resident CSR
// (LHPC_PLAN_DEVICE_INPUT); every decision (chunk cuts, segment offsets,
// pieces, ranges) stays the host code of lhpc_plan.cpp, fed the counts this
// pass produces, so the layout is byte-identical to the host build's
// (tests/test_gpu_spmv.py::test_device_input_layout_matches_host).
constexpr int kXtBuildMaxS = 4096;
// lhpc_plan.hpp xtile_wave_pos, on the device
__device__ __forceinline__ int64_t xtile_wave_pos_dev(int64_t i, int run, int vw) {
  const int64_t t = i / run, j = i % run, w = t / 64, l = t % 64, q = j / vw, r = j % vw;
  return w * 64 * run + (q * 64 + l) * vw + r;
}

// counts[c·S + s] = nonzeros of chunk c in tile s (LDS histogram per chunk)
__global__ __launch_bounds__(256) void k_xt_counts(const int32_t *__restrict__ ce, const int32_t *__restrict__ col,
                                                   int64_t W, int S, int32_t *__restrict__ counts) {
  __shared__ int32_t h[kXtBuildMaxS];
  const int64_t c = blockIdx.x;
  for (int s = threadIdx.x; s < S; s += blockDim.x) h[s] = 0;
  __syncthreads();
  const int e0 = ce[c], e1 = ce[c + 1];
  for (int k = e0 + static_cast<int>(threadIdx.x); k < e1; k += blockDim.x)
    atomicAdd(&h[static_cast<int>(col[k] / W)], 1);
  __syncthreads();
  for (int s = threadIdx.x; s < S; s += blockDim.x) counts[c * S + s] = h[s];
}

// One wave per chunk, its nonzeros in CSR order 64 at a time: a nonzero's
// slot in its (tile, chunk) segment is the segment's running count plus its
// rank among the step's lanes with the same tile (lanes matched by one
// ballot per tile-index bit) — the host scatter's stable order.  Writes
// col16 at the stream slot, and either perm (the slot's LDS offset) or the
// CSR-order iperm (flat position in the chunk's segment concatenation) in the
// wave-transposed run layout, with val in the same layout.
template <typename T, bool IP>
__global__ __launch_bounds__(64) void k_xt_scatter(
    const int32_t *__restrict__ ce, const int32_t *__restrict__ segoff, const int32_t *__restrict__ vbase,
    const int32_t *__restrict__ col, const T *__restrict__ val, int64_t W, int S, int sbits,
    uint16_t *__restrict__ col16, uint16_t *__restrict__ perm, uint16_t *__restrict__ ipt, T *__restrict__ valt) {
  __shared__ int32_t base[kXtBuildMaxS];  // segment start of (s, c)
  __shared__ int32_t cur[kXtBuildMaxS];   // entries placed so far
  __shared__ int32_t flat[kXtBuildMaxS];  // flat offset of the segment in the chunk
  const int64_t c = blockIdx.x;
  const int lane = threadIdx.x;
  constexpr int RUN = xt_run<T>(), VW = 16 / static_cast<int>(sizeof(T));
  for (int s = lane; s < S; s += 64) {
    base[s] = segoff[c * S + s];
    cur[s] = 0;
    flat[s] = segoff[(c + 1) * S + s] - segoff[c * S + s];  // length, scanned below
  }
  __syncthreads();
  if (IP && lane == 0) {  // exclusive scan of the lengths over the tiles (≤ 4096)
    int32_t f = 0;
    for (int s = 0; s < S; ++s) {
      const int32_t l = flat[s];
      flat[s] = f;
      f += l;
    }
  }
  __syncthreads();
  const int e0 = ce[c], e1 = ce[c + 1];
  const int64_t vb = vbase[c];
  for (int k0 = e0; k0 < e1; k0 += 64) {
    const int k = k0 + lane;
    const bool ok = k < e1;
    const int32_t cv = ok ? col[k] : 0;
    const int s = ok ? static_cast<int>(cv / W) : 0;
    uint64_t m = __ballot(ok);
    for (int b = 0; b < sbits; ++b) {
      const uint64_t bal = __ballot(ok && ((s >> b) & 1));
      m &= ((s >> b) & 1) ? bal : ~bal;
    }
    const uint64_t lt = (uint64_t{1} << lane) - 1;
    const int rank = __popcll(m & lt);
    const int before = ok ? cur[s] : 0;
    __builtin_amdgcn_wave_barrier();
    if (ok && rank == 0) cur[s] = before + __popcll(m);  // the lowest lane of each tile group
    __builtin_amdgcn_wave_barrier();
    if (ok) {
      const int i = k - e0;  // chunk position
      const int rel = before + rank;
      const int64_t g = static_cast<int64_t>(base[s]) + rel;
      col16[g] = static_cast<uint16_t>(cv - s * W);
      if constexpr (IP) {
        ipt[vb + xtile_wave_pos_dev(i, RUN, 8)] = static_cast<uint16_t>(flat[s] + rel);
      } else {
        perm[g] = static_cast<uint16_t>(xt_slot<T>(i));  // lhpc_plan.hpp xtile_slot(i, sizeof(T))
      }
      valt[vb + xtile_wave_pos_dev(i, RUN, VW)] = val[k];
    }
  }
}

// the gather's wave-coalesced store order (lhpc_plan.hpp xtile_gather_pos):
// inside each piece, every full 512-entry block of col16 from the piece start
// is permuted so that lane l's 8 entries are the stream positions its 16-B
// stores cover.  One workgroup (64 lanes) per piece.
__global__ __launch_bounds__(64) void k_xt_permute_blocks(const int32_t *__restrict__ pieces, int vw,
                                                          uint16_t *__restrict__ col16) {
  const int64_t g0 = pieces[3 * blockIdx.x], g1 = pieces[3 * blockIdx.x + 1];
  const int l = threadIdx.x;
  for (int64_t g = g0; g + 512 <= g1; g += 512) {
    uint16_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = col16[g + (k / vw) * 64 * vw + vw * l + k % vw];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) col16[g + 8 * l + k] = v[k];
    __syncthreads();
  }
}

// dev: col_idx and val are device pointers (LHPC_PLAN_DEVICE_INPUT; rp is a
// host copy of row_ptr): the O(nnz) passes run on the GPU
template <typename T>
int build_t(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, bool dev) {
  constexpr size_t tsz = sizeof(T);
  constexpr int M = XtRed<T, xt_red_blk<T>()>::M, RMAX = XtRed<T, xt_red_blk<T>()>::Rmax, RUN = xt_run<T>();
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, p->device) == hipSuccess) cus = prop.multiProcessorCount;
  // tile width: the LDS capacity XtTile<T>::W, narrowed for fp32 so that the
  // tile count is a whole multiple of the CUs when that adds ≤ 10% tiles
  // (C2: 245 → 256 tiles of 39063 columns): a cache-sized range's gather
  // round of one piece per tile then fills every CU.  fp64 (single range,
  // ≈ 2 pieces per CU) lost 3% with it (C3 489 → 512 tiles: 0.913 → 0.941 ms)
  int64_t W = XtTile<T>::W;
  {
    const int64_t s0 = (p->n_cols + W - 1) / W, s1 = (s0 + cus - 1) / cus * cus;
    // (never past build_xtile's 4096-tile cap: on a CU count that does not
    // divide 4096 the rounding could otherwise cost a plan its XTILE layout)
    bool narrow = sizeof(T) == 4 && s1 * 10 <= s0 * 11 && s1 <= 4096;
    if (const char *e = tuning_env("LHPC_XTILE_TW")) narrow = std::atoi(e) != 0;
    if (narrow && s1 > s0) W = (p->n_cols + s1 - 1) / s1;
  }
  // ≈ 2 gather workgroups per CU (one resident per CU: 160 KB of LDS each)
  // and ≥ 4 tiles' worth of stream per piece, so the tile load (W·T bytes)
  // stays ≤ 1/4 of a piece's col16 + xg traffic on small (per-rank) matrices
  const int64_t min_piece = 4 * W * static_cast<int64_t>(tsz) / (2 + static_cast<int64_t>(tsz));
  int64_t piece = std::max<int64_t>(min_piece, p->nnz / (2 * static_cast<int64_t>(cus)) + 1);
  const lhpc_options &o = p->opt;
  if (o.xtile_piece > 0) piece = std::max<int64_t>(8, o.xtile_piece);
  // reduce index stream: iperm (gather each CSR position's x from the flat
  // segment concatenation in LDS), else perm (scatter into CSR slots).  Round
  // 1 kept perm below 32 full chunks per CU (per-rank matrices at N ≥ 4);
  // with the reduce as it is now iperm is as fast or faster there too — same
  // box, local work of rank 0 (tools/explore_rank_reduce.py,
  // profiles/r04/rank_reduce.jsonl): fp32 W = 4 0.132 → 0.118 ms, W = 8
  // 0.0656 → 0.0653; fp64 W = 4 0.263 → 0.245, W = 8 0.125 → 0.118
  bool ip = true;
  if (o.xtile_reduce != LHPC_XTILE_REDUCE_AUTO) ip = o.xtile_reduce == LHPC_XTILE_REDUCE_IPERM;
  // the iperm reduce addresses xg with 32-bit buffer offsets: stream + tile
  // padding (≤ 8 per tile) + one piece of slack must stay below 2 GiB
  const int64_t n_tiles = (p->n_cols + W - 1) / W;
  const int64_t stream_max = p->nnz + 8 * n_tiles + 2 * M;
  if (stream_max * static_cast<int64_t>(tsz) >= (int64_t{1} << 31)) ip = false;
  p->xt_p = ip ? 3 : 1;
  // aligned segments (iperm only): each (tile, chunk) segment padded to 16 B
  // (≤ VW − 1 entries per segment, ≤ 3 per 4 nonzeros in the worst case)
  constexpr int VW = static_cast<int>(16 / tsz);
  bool al = false;
  if (o.xtile_align == LHPC_XTILE_ALIGN_UNITS) al = true;
  if (al && (!ip || (stream_max + (VW - 1) * std::min<int64_t>(p->nnz, n_tiles * (p->nnz / (M / 2) + 2))) *
                                static_cast<int64_t>(tsz) >= (int64_t{1} << 31)))
    al = false;
  // the fp32 aligned reduce with 8 segment-table entries per thread (S > 2048
  // tiles, n_cols > 84M) would spill a VGPR: packed segments there
  if (al && xtile_g<T>(static_cast<int>(std::min<int64_t>(n_tiles, 4096))) > 4) al = false;
  p->xt_al = al ? 1 : 0;
  // chunk cuts: at the last row start in the back M/32 of the window, else
  // mid-row (the row's pieces meet in k_xtile_fixup).  Per-chunk costs are
  // fixed, so full chunks matter on skewed rows: C4 has 19803 chunks when any
  // row start in the back half is taken, 18454 with the back M/32 (C2: 18316
  // either way); options.xtile_cut overrides (entries, 1..M)
  int cut = M / 32;
  if (o.xtile_cut > 0) cut = std::min(M, o.xtile_cut);
  // cache-sized ranges: K nnz-balanced row ranges, gathered and reduced in
  // turn, so that each range's xg (≈ 200 MB) is still in the 256 MB Infinity
  // Cache when its reduce reads it back.  fp32 only: each extra range re-reads
  // x (n_cols·T) in its gather.  Same box: C2 reduce 352 → 295
  // µs, gather 163 → 179 µs, call 523.5 → 483.8 µs at K = 3 (K = 4: 506.7);
  // C3 (fp64, K = 6: 200 MB ranges) 928 → 944 µs, so not for fp64 — until
  // the xg ring (round 6, same box, xtile_ranges = 1 / 3 / 4 / 6 / 8: C3
  // 0.908 / 0.943 / 0.995 / 0.868 / 0.902 ms): fp64 takes the ranges when its
  // plan can hold the ring (no user row splits, iperm reduce).
  // Only while each range still streams ≥ min_piece nonzeros per tile (fp64:
  // min_piece / 2 — its ring saves the 8-B xg write-back) and K ≤ 8: every
  // range re-loads all S tiles of x, so a wide x (n = 80M: 1954 tiles; n =
  // 150M: 3662) would spend more on tile loads than the cache saves — such
  // plans keep one range (the n = 150M plan took 23.6 ms with 8 ranges per part)
  int mall = 0;
  {
    const int64_t xg_bytes = p->nnz * static_cast<int64_t>(tsz);
    const int64_t k = (xg_bytes + (int64_t{200} << 20) - 1) / (int64_t{200} << 20);
    const int64_t tiles = (p->n_cols + W - 1) / W;
    // the xg ring: the plan's own cache ranges by default; user row ranges
    // only when asked for (xtile_ring = 2: the library's per-rank plans,
    // which gather and reduce range by range in order)
    const bool ring_ok = ip && !al && (p->split_rows.empty() ? o.xtile_ring != 1 : o.xtile_ring == 2);
    const int64_t need = tsz == 4 ? min_piece : min_piece / 2;
    if ((tsz == 4 || ring_ok) && xg_bytes > (int64_t{256} << 20) && k <= 8 &&
        p->nnz / k / std::max<int64_t>(1, tiles) >= need)
      mall = static_cast<int>(k);
  }
  if (o.xtile_ranges > 0) mall = o.xtile_ranges;
  // a row-range plan (user splits) whose xg exceeds the cache gets per-range
  // gather pieces for its own ranges (stage still gathers them all)
  const bool user_splits = !p->split_rows.empty();
  if (!p->split_rows.empty() && mall > 1) p->xt_mall = static_cast<int>(p->split_rows.size()) + 1;
  if (p->split_rows.empty() && mall > 1 && p->n_rows >= 2LL * mall) {
    std::vector<int64_t> cuts(static_cast<size_t>(mall) + 1);
    LHPC_TRY(lhpc_csr_partition_rows(rp.p, rp.bits, p->n_rows, mall, cuts.data()));
    for (int k = 1; k < mall; ++k)
      if (cuts[k] > 0 && cuts[k] < p->n_rows && (p->split_rows.empty() || cuts[k] > p->split_rows.back()))
        p->split_rows.push_back(cuts[k]);
    p->xt_mall = static_cast<int>(p->split_rows.size()) + 1;
  }
  XtileHost xt;
  // device-side O(nnz) buffers (dev only): chunk starts, segment starts, run bases
  struct DevTmp {
    void *a = nullptr;
    ~DevTmp() {
      if (a) (void)hipFree(a);
    }
  } d_ce, d_segoff, d_vbase, d_counts;
  if (dev) {
    if (al) return LHPC_ERR_UNSUPPORTED;  // aligned segments: host build only
    LHPC_TRY(xtile_plan_chunks(rp.p, rp.bits, nullptr, p->n_rows, p->n_cols, W, M, RMAX, static_cast<int>(tsz),
                               p->split_rows.data(), static_cast<int>(p->split_rows.size()), ip, cut, xt, 1));
    const int64_t S = xt.S, C = xt.n_chunks;
    if (S > kXtBuildMaxS) return LHPC_ERR_UNSUPPORTED;
    LHPC_HIP_TRY(hipMalloc(&d_ce.a, xt.ce.size() * 4));
    LHPC_HIP_TRY(hipMemcpy(d_ce.a, xt.ce.data(), xt.ce.size() * 4, hipMemcpyHostToDevice));
    if (C > 0) {
      LHPC_HIP_TRY(hipMalloc(&d_counts.a, static_cast<size_t>(C * S) * 4));
      hipLaunchKernelGGL(k_xt_counts, dim3(static_cast<unsigned>(C)), dim3(256), 0, nullptr,
                         static_cast<const int32_t *>(d_ce.a), col_idx, W, static_cast<int>(S),
                         static_cast<int32_t *>(d_counts.a));
      LHPC_HIP_TRY(hipGetLastError());
      LHPC_HIP_TRY(hipMemcpy(xt.segoff.data() + S, d_counts.a, static_cast<size_t>(C * S) * 4, hipMemcpyDeviceToHost));
    }
    std::vector<int64_t> tbase;
    LHPC_TRY(xtile_plan_offsets(xt, tbase));
    xtile_plan_pieces(xt, tbase, piece);
  } else {
    LHPC_TRY(build_xtile(rp.p, rp.bits, col_idx, p->n_rows, p->n_cols, W, M, RMAX, piece, static_cast<int>(tsz),
                         p->split_rows.data(), static_cast<int>(p->split_rows.size()), ip, cut, xt, al ? VW : 1));
  }
  p->kernel = LHPC_KERNEL_XTILE;
  p->rp64 = 0;
  p->S = xt.S;
  p->xs_width = W;
  p->xt_C = xt.n_chunks;
  p->xt_pieces = static_cast<int64_t>(xt.pieces.size() / 3);
  p->xt_cont = static_cast<int64_t>(xt.cont.size());
  p->xt_total = xt.total;
  // phase-A tables (options.xtile_pretable): iperm
  // plans without aligned segments, G = 1.  Default for fp64 only — same box,
  // two runs each: C3 reduce 89.9 → 85.3 µs per range (its 16-wave scan was
  // 2.3K of 27.8K cycles per chunk), C2 88.1 → 89.4 µs (the tables' extra
  // 2 KB per chunk outweigh an 8-wave scan)
  const bool pre = ip && !al && xtile_g<T>(xt.S) == 1 &&
                   (o.xtile_pretable == 2 || (o.xtile_pretable == 0 && sizeof(T) == 8));
  p->xt_pre = pre ? 1 : 0;
  p->xt_lds = xtile_lds_bytes_g<T>(xt.S, xtile_g<T>(xt.S), pre);
#ifdef LHPC_XT_LDS_TOTAL  // A/B build only: reduce blocks padded to this many bytes of LDS (fewer per CU)
  if (sizeof(T) == 4) p->xt_lds = std::max<size_t>(p->xt_lds, LHPC_XT_LDS_TOTAL);
#endif
  if (o.xtile_steps > 0) {
    const int u = o.xtile_steps;
    p->xt_u = u <= 2 ? 2 : u < 8 ? 4 : u < 16 ? 8 : 16;
  }
  // non-temporal xg stores when the xg of a single-range plan exceeds the 256
  // MB Infinity Cache anyway (same box, two runs each: C3 918.6 → 908.8 µs
  // median); cache-sized ranges need their xg to stay there (C2 with them
  // non-temporal: 473 → 536 µs)
  p->xt_nt = p->xt_mall <= 1 && p->nnz * static_cast<int64_t>(tsz) > (int64_t{256} << 20) ? 1 : 0;
  if (o.xtile_store != LHPC_STORE_AUTO) p->xt_nt = o.xtile_store == LHPC_STORE_NT ? 1 : 0;
  const void *rfn = xtile_reduce_fn<T>(xtile_g<T>(xt.S), ip, al, pre);
  if (!rfn) return LHPC_ERR_UNSUPPORTED;  // more tiles than the reduce's segment table holds
  LHPC_HIP_TRY(hipFuncSetAttribute(rfn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(p->xt_lds)));
  const int64_t n_rows = p->n_rows, C = xt.n_chunks;
  auto up = [&](void **d, const void *h, size_t n) -> int {
    LHPC_TRY(dmalloc(d, n, p->bytes));
    if (n && h) LHPC_HIP_TRY(hipMemcpy(*d, h, n, hipMemcpyHostToDevice));
    return LHPC_OK;
  };
  std::vector<int32_t> rp32(static_cast<size_t>(n_rows + 1));
  for (int64_t i = 0; i <= n_rows; ++i) rp32[static_cast<size_t>(i)] = static_cast<int32_t>(rp[i]);
  LHPC_TRY(up(&p->d_row_ptr, rp32.data(), rp32.size() * 4));
  // val (and iperm) in the wave-transposed run layout, each chunk padded to
  // whole wave regions, plus one region of zeros (an empty chunk reads it)
  std::vector<int32_t> vbase;
  std::unique_ptr<unsigned char[]> valt;
  std::unique_ptr<uint16_t[]> ipt;
  size_t nrun = 0;
  if (dev) {
    // run bases as xtile_transpose_runs; the runs themselves come from
    // k_xt_scatter (val zero-padded, iperm padded with the zero slot M)
    std::vector<int64_t> vb(static_cast<size_t>(C) + 1, 0);
    const int64_t reg = 64 * RUN;
    for (int64_t c = 0; c < C; ++c) vb[c + 1] = vb[c] + (xt.ce[c + 1] - xt.ce[c] + reg - 1) / reg * reg;
    if (vb[C] + reg >= INT32_MAX) return LHPC_ERR_UNSUPPORTED;
    vbase.assign(vb.begin(), vb.end());
    nrun = static_cast<size_t>(vbase[C]) + 64 * RUN;
    p->xt_nrun = static_cast<int64_t>(nrun);
    LHPC_TRY(dmalloc(&p->d_val, nrun * tsz, p->bytes));
    LHPC_HIP_TRY(hipMemset(p->d_val, 0, nrun * tsz));
  } else {
    LHPC_TRY(xtile_transpose_runs(xt, val, tsz, RUN, 64 * RUN, vbase, valt, ipt));
    nrun = static_cast<size_t>(vbase[C]) + 64 * RUN;
    p->xt_nrun = static_cast<int64_t>(nrun);
    LHPC_TRY(up(&p->d_val, valt.get(), nrun * tsz));
    valt.reset();
  }
  {
    std::vector<int32_t> cd(static_cast<size_t>(8 * C + 8), 0);  // {e0, e1, r0, r1, vbase, 0, 0, 0}
    for (int64_t c = 0; c < C; ++c) {
      cd[8 * c] = xt.ce[c];
      cd[8 * c + 1] = xt.ce[c + 1];
      cd[8 * c + 2] = xt.cr[c];
      cd[8 * c + 3] = xt.cr[c + 1];
      cd[8 * c + 4] = vbase[c];
    }
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_cdesc), cd.data(), cd.size() * 4));
  }
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_cr), xt.cr.data(), xt.cr.size() * 4));
  if (p->xt_mall > 1) {
    // one gather round per range: ≈ one piece per (tile, range) part, so each
    // range loads every tile once (only one 160-KB gather block fits a CU)
    int64_t rpn = std::max<int64_t>(min_piece, p->nnz / p->xt_mall / static_cast<int64_t>(cus) * 5 / 4 + 1);
    if (o.xtile_range_piece > 0) rpn = std::max<int64_t>(8, o.xtile_range_piece);
    // the xg ring (options.xtile_ring): the plan's own cache
    // ranges; user row ranges only with xtile_ring = 2 (lhpc_spmv_stage would
    // gather every range into the one ring: a ring plan refuses it)
    p->xt_ring = ip && !al && (user_splits ? o.xtile_ring == 2 : o.xtile_ring != 1) ? 1 : 0;
    if (p->xt_ring) {
      xtile_ring_pieces(xt, rpn, p->xt_rpc);
      p->xt_ring_len = xt.ring_len;
      p->xt_hrow = xt.hrow;
    } else {
      xtile_range_pieces(xt, rpn, p->xt_rpc);
    }
    p->xt_pieces = static_cast<int64_t>(xt.pieces.size() / 3);
  }
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_pieces), xt.pieces.data(), xt.pieces.size() * 4));
  if (p->xt_ring) LHPC_TRY(up(reinterpret_cast<void **>(&p->d_pext), xt.pext.data(), xt.pext.size() * 4));
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_cont), xt.cont.data(), xt.cont.size() * 4));
  if (dev) {
    // col16 and perm / iperm + val runs on the device, then the gather-store
    // permutation of col16 inside every piece
    const int64_t S = xt.S;
    LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_col16), static_cast<size_t>(xt.total) * 2, p->bytes));
    LHPC_HIP_TRY(hipMemset(p->d_col16, 0, static_cast<size_t>(std::max<int64_t>(xt.total, 1)) * 2));
    if (ip) {
      LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_perm), nrun * 2, p->bytes));
      LHPC_HIP_TRY(hipMemsetD16(reinterpret_cast<hipDeviceptr_t>(p->d_perm), static_cast<unsigned short>(M), nrun));
    } else {
      LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_perm), static_cast<size_t>(xt.total + 2) * 2, p->bytes));
      LHPC_HIP_TRY(hipMemset(p->d_perm, 0, static_cast<size_t>(xt.total + 2) * 2));
      const uint16_t spare[2] = {static_cast<uint16_t>(M), static_cast<uint16_t>(M)};
      LHPC_HIP_TRY(hipMemcpy(p->d_perm + xt.total, spare, 4, hipMemcpyHostToDevice));
    }
    if (C > 0) {
      LHPC_HIP_TRY(hipMalloc(&d_segoff.a, xt.segoff.size() * 4));
      LHPC_HIP_TRY(hipMemcpy(d_segoff.a, xt.segoff.data(), xt.segoff.size() * 4, hipMemcpyHostToDevice));
      LHPC_HIP_TRY(hipMalloc(&d_vbase.a, vbase.size() * 4));
      LHPC_HIP_TRY(hipMemcpy(d_vbase.a, vbase.data(), vbase.size() * 4, hipMemcpyHostToDevice));
      int sbits = 0;
      while ((int64_t{1} << sbits) < S) ++sbits;
      if (ip)
        hipLaunchKernelGGL((k_xt_scatter<T, true>), dim3(static_cast<unsigned>(C)), dim3(64), 0, nullptr,
                           static_cast<const int32_t *>(d_ce.a), static_cast<const int32_t *>(d_segoff.a),
                           static_cast<const int32_t *>(d_vbase.a), col_idx, static_cast<const T *>(val), W,
                           static_cast<int>(S), sbits, p->d_col16, nullptr, p->d_perm, static_cast<T *>(p->d_val));
      else
        hipLaunchKernelGGL((k_xt_scatter<T, false>), dim3(static_cast<unsigned>(C)), dim3(64), 0, nullptr,
                           static_cast<const int32_t *>(d_ce.a), static_cast<const int32_t *>(d_segoff.a),
                           static_cast<const int32_t *>(d_vbase.a), col_idx, static_cast<const T *>(val), W,
                           static_cast<int>(S), sbits, p->d_col16, p->d_perm, nullptr, static_cast<T *>(p->d_val));
      LHPC_HIP_TRY(hipGetLastError());
    }
    const int64_t np = static_cast<int64_t>(xt.pieces.size() / 3);
    if (np > 0) {
      hipLaunchKernelGGL(k_xt_permute_blocks, dim3(static_cast<unsigned>(np)), dim3(64), 0, nullptr, p->d_pieces,
                         static_cast<int>(16 / tsz), p->d_col16);
      LHPC_HIP_TRY(hipGetLastError());
    }
    LHPC_HIP_TRY(hipDeviceSynchronize());
  } else {
    xtile_permute_gather_blocks(xt, static_cast<int>(16 / tsz));
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_col16), xt.col16.get(), static_cast<size_t>(xt.total) * 2));
  }
  if (pre) {  // the reduce's phase-A tables in place of the segment table (seg = bt, seghi = base_ne)
    std::vector<uint32_t> pbt;
    std::vector<int32_t> pbne;
    xtile_phase_tables(xt, pbt, pbne);
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_seg), pbt.data(), pbt.size() * 4));
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_seghi), pbne.data(), pbne.size() * 4));
    p->xt_seg_n = static_cast<int64_t>(pbt.size());
    p->xt_seghi_n = static_cast<int64_t>(pbne.size());
  } else {
    std::vector<uint32_t> seg;
    std::vector<int32_t> seghi;
    xtile_segment_table(xt, seg, seghi);
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_seg), seg.data(), seg.size() * 4));
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_seghi), seghi.data(), seghi.size() * 4));
    p->xt_seg_n = static_cast<int64_t>(seg.size());
    p->xt_seghi_n = static_cast<int64_t>(seghi.size());
  }
  if (dev) {
    // built above
  } else if (ip) {
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_perm), ipt.get(), nrun * 2));
  } else {
    // one sentinel entry past the stream: the reduce loads it for positions
    // past m, and its perm is the spare LDS slot M
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_perm), nullptr, static_cast<size_t>(xt.total + 2) * 2));
    if (xt.total) LHPC_HIP_TRY(hipMemcpy(p->d_perm, xt.perm.get(), static_cast<size_t>(xt.total) * 2, hipMemcpyHostToDevice));
    const uint16_t spare[2] = {static_cast<uint16_t>(M), static_cast<uint16_t>(M)};
    LHPC_HIP_TRY(hipMemcpy(p->d_perm + xt.total, spare, 4, hipMemcpyHostToDevice));
  }
  LHPC_TRY(up(&p->d_xg, nullptr, static_cast<size_t>((p->xt_ring ? xt.ring_len : xt.total) + 2) * tsz));
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_carry), nullptr, static_cast<size_t>(2 * C + 2) * 8));
  LHPC_HIP_TRY(hipMemset(p->d_carry, 0, static_cast<size_t>(2 * C + 2) * 8));
  if (!p->split_rows.empty()) {
    const size_t K = p->split_rows.size() + 1;
    p->xt_srow.assign(1, 0);
    p->xt_srow.insert(p->xt_srow.end(), p->split_rows.begin(), p->split_rows.end());
    p->xt_srow.push_back(n_rows);
    p->xt_src.assign(xt.rchunk.begin(), xt.rchunk.end());
    p->xt_sco.assign(K + 1, 0);
    for (size_t k = 0; k <= K; ++k)
      p->xt_sco[k] = std::lower_bound(xt.cont.begin(), xt.cont.end(), static_cast<int32_t>(p->xt_src[k])) -
                     xt.cont.begin();
  }
  return LHPC_OK;
}

}  // namespace

template <typename T>
int launch_mall(const lhpc_spmv_plan *p, const void *x, T *y, hipStream_t s) {
  for (int k = 0; k < p->xt_mall; ++k) {
    LHPC_TRY(launch_gather<T>(p, x, s, p->xt_rpc[k], p->xt_rpc[k + 1]));
    LHPC_TRY(launch_reduce<T>(p, p->xt_src[k], p->xt_src[k + 1], 0, 0, y, s, p->xt_ring ? k : -1));
  }
  // one fix-up for every range's cut rows (their carries stay in place)
  return launch_reduce<T>(p, p->xt_C, p->xt_C, 0, p->xt_cont, y, s);
}

int xtile_launch(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  if (p->n_rows == 0) return LHPC_OK;
  if (p->xt_mall > 1)
    return p->dtype == LHPC_F32 ? launch_mall<float>(p, x, static_cast<float *>(y), s)
                                : launch_mall<double>(p, x, static_cast<double *>(y), s);
  if (p->dtype == LHPC_F32) {
    LHPC_TRY(launch_gather<float>(p, x, s));
    return launch_reduce<float>(p, 0, p->xt_C, 0, p->xt_cont, static_cast<float *>(y), s);
  }
  LHPC_TRY(launch_gather<double>(p, x, s));
  return launch_reduce<double>(p, 0, p->xt_C, 0, p->xt_cont, static_cast<double *>(y), s);
}

// lhpc_spmv_stage: the gather of a split plan; lhpc_spmv_range: range k's
// reduce + fix-up into y_k (row xt_srow[k] at y_k[0]).  xtile_range_gather:
// range k's gather alone (plans with per-range pieces; ranges gathered in
// order 0, 1, … — a range's first ≤ 7 entries come from the one before).
int xtile_stage(const lhpc_spmv_plan *p, const void *x, hipStream_t s) {
  return p->dtype == LHPC_F32 ? launch_gather<float>(p, x, s) : launch_gather<double>(p, x, s);
}

int xtile_range_gather(const lhpc_spmv_plan *p, const void *x, int k, hipStream_t s) {
  if (p->xt_rpc.empty() || k < 0 || k + 2 > static_cast<int>(p->xt_rpc.size())) return LHPC_ERR_UNSUPPORTED;
  return p->dtype == LHPC_F32 ? launch_gather<float>(p, x, s, p->xt_rpc[k], p->xt_rpc[k + 1])
                              : launch_gather<double>(p, x, s, p->xt_rpc[k], p->xt_rpc[k + 1]);
}

int xtile_range(const lhpc_spmv_plan *p, int k, void *yk, hipStream_t s) {
  const int64_t c0 = p->xt_src[k], c1 = p->xt_src[k + 1], n0 = p->xt_sco[k], n1 = p->xt_sco[k + 1];
  const int ring = p->xt_ring ? k : -1;  // a ring plan: range k was the last one gathered
  if (p->dtype == LHPC_F32)
    return launch_reduce<float>(p, c0, c1, n0, n1, static_cast<float *>(yk) - p->xt_srow[k], s, ring);
  return launch_reduce<double>(p, c0, c1, n0, n1, static_cast<double *>(yk) - p->xt_srow[k], s, ring);
}

int xtile_part_of_tile(int64_t tile, int64_t tile_width, int64_t n_cols, const int64_t *col_end, int n_parts) {
  const int64_t last = std::min((tile + 1) * tile_width, n_cols);  // exclusive end of the tile's columns
  for (int j = 0; j < n_parts; ++j)
    if (col_end[j] >= last) return j;
  return n_parts - 1;
}

int xtile_column_parts(lhpc_spmv_plan *p, const int64_t *col_end, int n_parts) {
  if (p->kernel != LHPC_KERNEL_XTILE || !p->xt_rpc.empty() || n_parts < 1) return LHPC_ERR_UNSUPPORTED;
  for (int j = 0; j < n_parts; ++j)
    if (col_end[j] < 0 || (j > 0 && col_end[j] < col_end[j - 1])) return LHPC_ERR_INVALID_ARG;
  if (col_end[n_parts - 1] < p->n_cols) return LHPC_ERR_INVALID_ARG;
  const int64_t np = p->xt_pieces;
  std::vector<int32_t> pc(static_cast<size_t>(3 * np)), out;
  out.reserve(pc.size());
  LHPC_HIP_TRY(hipSetDevice(p->device));
  if (np) LHPC_HIP_TRY(hipMemcpy(pc.data(), p->d_pieces, pc.size() * 4, hipMemcpyDeviceToHost));
  // stable partition by part: the pieces are in ascending runs of 8 tiles,
  // so each part keeps the run order (and its same-XCD tile interleave)
  p->xt_cpf.assign(1, 0);
  for (int j = 0; j < n_parts; ++j) {
    for (int64_t q = 0; q < np; ++q)
      if (xtile_part_of_tile(pc[3 * q + 2], p->xs_width, p->n_cols, col_end, n_parts) == j)
        out.insert(out.end(), pc.begin() + 3 * q, pc.begin() + 3 * q + 3);
    p->xt_cpf.push_back(static_cast<int64_t>(out.size() / 3));
  }
  if (p->d_pieces_cp) (void)hipFree(p->d_pieces_cp);
  p->d_pieces_cp = nullptr;
  LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_pieces_cp), out.size() * 4, p->bytes));
  if (!out.empty()) LHPC_HIP_TRY(hipMemcpy(p->d_pieces_cp, out.data(), out.size() * 4, hipMemcpyHostToDevice));
  p->xt_cpe.assign(col_end, col_end + n_parts);
  return LHPC_OK;
}

int xtile_stage_part(const lhpc_spmv_plan *p, const void *x, int j, hipStream_t s) {
  if (p->xt_cpf.empty() || j < 0 || j + 2 > static_cast<int>(p->xt_cpf.size())) return LHPC_ERR_INVALID_ARG;
  return p->dtype == LHPC_F32 ? launch_gather<float>(p, x, s, p->xt_cpf[j], p->xt_cpf[j + 1], p->d_pieces_cp)
                              : launch_gather<double>(p, x, s, p->xt_cpf[j], p->xt_cpf[j + 1], p->d_pieces_cp);
}

int xtile_build(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz) {
  return tsz == 4 ? build_t<float>(p, rp, col_idx, val, false) : build_t<double>(p, rp, col_idx, val, false);
}

int xtile_build_device(lhpc_spmv_plan *p, RowPtrView rp_host, const int32_t *d_col, const void *d_val, size_t tsz) {
  return tsz == 4 ? build_t<float>(p, rp_host, d_col, d_val, true) : build_t<double>(p, rp_host, d_col, d_val, true);
}

}  // namespace lhpc

#ifdef LHPC_XT_STAMPS
// diagnostic build: copy the reduce's phase stamps (uint64 [blocks][10]) to host
extern "C" int lhpc_probe_xtile_stamps(void *out, int64_t n) {
  try {
    if (n > (1 << 22)) n = 1 << 22;
    LHPC_HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(lhpc::g_xt_stamps), static_cast<size_t>(n) * 8, 0,
                                     hipMemcpyDeviceToHost));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}
extern "C" int lhpc_probe_xtile_stamps_clear(void) {
  try {
    static uint64_t zero[1 << 16];
    for (int64_t o = 0; o < (1 << 22); o += 1 << 16)
      LHPC_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(lhpc::g_xt_stamps), zero, sizeof(zero), static_cast<size_t>(o) * 8,
                                     hipMemcpyHostToDevice));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}
#endif
