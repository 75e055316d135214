// lhpc_sort.hip — LSD radix sort (uint32 keys; uint64 keys + uint32 values) and
// COO→CSR assembly for gfx950.
//
// Reference behaviour: sort::gpu::radix::radix_sort
// (lib/gpu/radix_gpu/src/radix_sort_gpu.cpp:24-29 → cuda_radix_sort_v4.cu:17-242)
// sorts a uint32 vector in place with four 8-bit LSD passes; the CPU twin
// sort::radix::radix_sort (lib/sort/radix_cpu/include/radix_sort_cpu.hpp:320-331)
// is the same LSD counting sort.  Sorted output is unique for keys, and for
// (key, value) pairs this sort is stable, so every result is bit-exact
// against a stable CPU sort.
//
// MI355X design (not a port of the reference's hierarchical 1024-tile scan):
//  * per 8-bit pass: upsweep (per-block digit histogram, block-major counts),
//    scan (one workgroup per digit: per-block exclusive prefixes + digit
//    totals), downsweep;
//  * even-share grid of 16 × the resident downsweep blocks: each block walks
//    its own run of TILE-key sub-tiles in order (1024-thread blocks, one per
//    CU: 20480 u32 keys, 16384 u32 or u64 pairs), so the per-block histogram
//    table stays small;
//  * downsweep ranks stably inside a sub-tile with a wave64 match-any
//    (8 ballots per key → peer mask; rank = popcount(peers & lanes below)),
//    per-wave running digit counters in LDS, then reorders the sub-tile in
//    LDS by digit so the global scatter writes contiguous digit runs;
//  * only bits [begin_bit, end_bit) are used (partial last digit masked).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "lhpc_common.hpp"

namespace lhpc {
namespace {

constexpr int kSortThreads = 256;
constexpr int kSortMaxResident = 2048;  // resident-block cap (and fallback if occupancy query fails)

// a & ~(b ^ c) as one gfx950 v_bitop3 (LUT index = a·4 + b·2 + c: rows 4
// and 7).  Device pass only: the host pass's check of the builtin would drop
// the kernels' host stubs (see lhpc_spmv_xtile.hip, aligned segments)
__device__ __forceinline__ uint32_t and_xnor(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x90);
#else
  return a & ~(b ^ c);
#endif
}

template <typename K>
__device__ __forceinline__ uint32_t digit_of(K k, int shift, uint32_t mask) {
  return static_cast<uint32_t>(k >> shift) & mask;
}

// Upsweep: digit histogram of the block's sub-tiles → counts[b·256 + d].
// 32-bit keys stream as LHPC_SORT_UP_Q 16-B non-temporal loads per thread and
// step (round 5, four: same box, 350.6 → 327.6 µs per 500M-key
// pass — 16 sub-histograms per block against LDS-atomic conflicts, and no
// atomics at all (timing only), both left it at 342–350 µs, so the key
// stream, not the atomics, bounds it); 64-bit keys four 8-B loads.
template <typename K, int TILE>
__global__ __launch_bounds__(kSortThreads) void k_radix_upsweep(const K *__restrict__ keys, int64_t n,
                                                                int shift, uint32_t mask, int64_t per_block,
                                                                uint32_t *__restrict__ counts, int vec16) {
  __shared__ uint32_t hist[4][256];
  const int t = threadIdx.x, w = t / kWave;
  for (int i = t; i < 4 * 256; i += kSortThreads) (&hist[0][0])[i] = 0;
  __syncthreads();
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * per_block * TILE;
  const int64_t b1 = std::min<int64_t>(n, b0 + per_block * TILE);
  int64_t i = b0;
  if constexpr (sizeof(K) == 4) {
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
// (eight 16-B loads per thread and step: 366 → 363 µs per 500M-key pass,
// two : 375; profiles/r06/ab_sort2/upsweep)
#ifndef LHPC_SORT_UP_Q  // A/B builds: 16-B loads per thread and step
#define LHPC_SORT_UP_Q 8
#endif
    constexpr int UQ = LHPC_SORT_UP_Q;
    constexpr int STEP = 4 * UQ * kSortThreads;
    // vec16 (host: keys 16-B aligned; a caller's key pointer may be 4-B
    // aligned only, e.g. a slice t[1:]): b0 is a multiple of TILE, so every
    // 16-B load is aligned; otherwise the scalar loop below takes every key
    for (; vec16 && i + STEP <= b1; i += STEP) {
      const u32x4v *p = reinterpret_cast<const u32x4v *>(keys + i) + t;
      u32x4v v[UQ];
#pragma unroll
      for (int q = 0; q < UQ; ++q) v[q] = __builtin_nontemporal_load(p + q * kSortThreads);
#pragma unroll
      for (int q = 0; q < UQ; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) atomicAdd(&hist[w][digit_of(static_cast<K>(v[q][e]), shift, mask)], 1u);
    }
  } else {
    // 64-bit keys: four 16-B non-temporal loads (two keys each) per thread
    // and step on 16-B aligned keys (round 6: 150M-pair COO sort, 240 → 212
    // µs per pass against four 8-B loads)
    typedef uint64_t u64x2v __attribute__((ext_vector_type(2)));
    constexpr int STEP8 = 8 * kSortThreads;
    for (; vec16 && i + STEP8 <= b1; i += STEP8) {
      const u64x2v *p = reinterpret_cast<const u64x2v *>(keys + i) + t;
      u64x2v v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = __builtin_nontemporal_load(p + q * kSortThreads);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 2; ++e) atomicAdd(&hist[w][digit_of(static_cast<K>(v[q][e]), shift, mask)], 1u);
    }
    for (; i + 4 * kSortThreads <= b1; i += 4 * kSortThreads) {
      const K k0 = keys[i + t], k1 = keys[i + kSortThreads + t], k2 = keys[i + 2 * kSortThreads + t],
              k3 = keys[i + 3 * kSortThreads + t];
      atomicAdd(&hist[w][digit_of(k0, shift, mask)], 1u);
      atomicAdd(&hist[w][digit_of(k1, shift, mask)], 1u);
      atomicAdd(&hist[w][digit_of(k2, shift, mask)], 1u);
      atomicAdd(&hist[w][digit_of(k3, shift, mask)], 1u);
    }
  }
  for (i += t; i < b1; i += kSortThreads) atomicAdd(&hist[w][digit_of(keys[i], shift, mask)], 1u);
  __syncthreads();
  counts[static_cast<int64_t>(blockIdx.x) * 256 + t] = hist[0][t] + hist[1][t] + hist[2][t] + hist[3][t];
}

// Block-wide exclusive scan of one value per thread (NW waves: 256 threads =
// 4); returns the total.  DPP scan inside each wave, the wave totals through
// LDS: two barriers (the Hillis-Steele form took 16 per call, and the
// downsweep runs two scans per 4096-key sub-tile).
// TRAIL = false: no closing barrier (the caller's next use of tmp is behind
// barriers of its own).
template <int NW = 4, bool TRAIL = true>
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *tmp /*[≥NW]*/, uint32_t &total) {
  const int t = threadIdx.x, w = t / kWave;
  const uint32_t inc = static_cast<uint32_t>(wave_incl_scan(static_cast<int>(v)));  // modular add: same bits
  if ((t & (kWave - 1)) == kWave - 1) tmp[w] = inc;
  __syncthreads();
  uint32_t off = 0, all = 0;
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const uint32_t tj = tmp[j];
    off += j < w ? tj : 0u;
    all += tj;
  }
  total = all;
  if constexpr (TRAIL) __syncthreads();  // tmp is reused by the caller's next scan
  return off + inc - v;
}
__device__ __forceinline__ uint32_t block_exscan256(uint32_t v, uint32_t *tmp, uint32_t &total) {
  return block_exscan<4>(v, tmp, total);
}

// Scan: one workgroup per digit d.  counts[b][d] → exclusive prefix over
// blocks (in place); totals[d] = Σ_b counts[b][d].  (The digit bases — the
// exclusive prefix of totals over digits — are formed by every downsweep block
// from the 256 totals.)
__global__ __launch_bounds__(kSortThreads) void k_radix_scan(uint32_t *__restrict__ counts, int nblocks,
                                                             uint32_t *__restrict__ totals) {
  __shared__ uint32_t tmp[256];
  const int d = blockIdx.x, t = threadIdx.x;
  uint32_t carry = 0;
  for (int b0 = 0; b0 < nblocks; b0 += kSortThreads * 4) {
    uint32_t c[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = b0 + t * 4 + j;
      c[j] = b < nblocks ? counts[static_cast<int64_t>(b) * 256 + d] : 0u;
      s += c[j];
    }
    uint32_t total;
    uint32_t run = carry + block_exscan256(s, tmp, total);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = b0 + t * 4 + j;
      if (b < nblocks) counts[static_cast<int64_t>(b) * 256 + d] = run;
      run += c[j];
    }
    carry += total;
  }
  if (t == 0) totals[d] = carry;
}

// wave64 match-any on an 8-bit digit: the lanes whose digit equals mine, one
// ballot per digit bit.  dm = 0 / all-ones from the bit by one signed
// bitfield extract, kept opaque (inline asm) so the compiler does not derive
// the ballot condition by a second shift of its own; the ballot is
// v_cmp(dm ≠ 0) and the mask update peers &= ~(ballot ^ dm) one v_bitop3 per
// half: 4 VALU per bit (5 when the compiler re-derived the condition).
__device__ __forceinline__ uint64_t match_any8(uint32_t d) {
  uint32_t plo = ~0u, phi = ~0u;
#pragma unroll
  for (int bit = 0; bit < 8; ++bit) {
    uint32_t dm;
#if defined(__HIP_DEVICE_COMPILE__)
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(dm) : "v"(d), "i"(bit));
#else
    dm = (d >> bit) & 1u ? ~0u : 0u;
#endif
    const uint64_t bal = __ballot(dm != 0u);
    plo = and_xnor(plo, static_cast<uint32_t>(bal), dm);
    phi = and_xnor(phi, static_cast<uint32_t>(bal >> 32), dm);
  }
  return (static_cast<uint64_t>(phi) << 32) | plo;
}

// Downsweep: stable rank within each sub-tile, LDS reorder, coalesced scatter.
// Sub-tile layout: wave w owns keys [w·IPT·64, (w+1)·IPT·64) of the sub-tile,
// visited as IPT rounds of 64 consecutive keys — so (wave, round, lane)
// order is the input order, which makes the rank stable.  Per round a
// match-any gives the lanes of equal digit; rank = the wave's running counter
// of that digit (LDS) + the peers below; the lowest peer advances the
// counter.  The digit offsets are folded once per sub-tile (wave prefix +
// sub-tile start into the wave counters; global base − sub-tile start into
// gofs), so the reorder and the scatter read one LDS word per key; the global
// base of digit t lives in thread t's register; full sub-tiles load and store
// without bounds checks; one barrier fewer per sub-tile than reading two
// offset tables (C2-sized sort, same box, three runs each: 9.04 → 8.91 ms).
// BT threads per block (NW = BT / 64 waves); threads t < 256 own digit t.
// SR (pairs): keys and values reordered one after the other through the one
// LDS buffer, so a sub-tile of 8-B keys needs TILE × 8 B of LDS instead of
// TILE × 12; each sorted position's digit is kept as a byte (dg) for the
// values' scatter, and the wave counters are 16-bit (< TILE ≤ 65536) to make
// room for it.
#ifdef LHPC_SORT_WPE  // A/B builds: waves per SIMD the downsweep's registers must allow
#define LHPC_SORT_DS_ATTR __attribute__((amdgpu_waves_per_eu(LHPC_SORT_WPE)))
#else
#define LHPC_SORT_DS_ATTR
#endif
template <typename K, bool HAS_V, int IPT, bool PF = true, int BT = kSortThreads, bool SR = false>
__global__ __launch_bounds__(BT) LHPC_SORT_DS_ATTR void k_radix_downsweep(
    const K *__restrict__ kin, K *__restrict__ kout, const uint32_t *__restrict__ vin, uint32_t *__restrict__ vout,
    int64_t n, int shift, uint32_t mask, int64_t per_block, const uint32_t *__restrict__ counts,
    const uint32_t *__restrict__ totals) {
  constexpr int TILE = IPT * BT;
  constexpr int WSEG = IPT * kWave;
  constexpr int NW = BT / kWave;
  static_assert(BT % 256 == 0, "threads t < 256 own the digits");
  static_assert(TILE <= 65536, "16-bit ranks");
  __shared__ K sk[TILE];
  static_assert(!SR || (HAS_V && !PF), "SR: pairs without the prefetch");
  __shared__ uint32_t sv[HAS_V && !SR ? TILE : 1];
  __shared__ std::conditional_t<SR, uint16_t, uint32_t> wcnt[NW][256];
  __shared__ uint8_t dg[SR ? TILE : 1];
  __shared__ uint32_t gofs[256];
  __shared__ uint32_t tmp[NW];
  const int t = threadIdx.x, w = t / kWave, lane = t & (kWave - 1);
  const bool own = BT == 256 || t < 256;  // thread t owns digit t
  uint32_t gb;  // thread t: global output position of digit t's next key
  {
    uint32_t all;
    gb = block_exscan<NW>(own ? totals[t] : 0u, tmp, all) +
         (own ? counts[static_cast<int64_t>(blockIdx.x) * 256 + t] : 0u);
  }
  const int64_t first = static_cast<int64_t>(blockIdx.x) * per_block;
  const int64_t ntiles = (n + TILE - 1) / TILE;
  const int64_t last = std::min<int64_t>(ntiles, first + per_block);
  K key[IPT];
  uint32_t val[IPT];
  // SR loads the values only after the keys' reorder (they are not live
  // through the rank and the scan)
  auto load_tile = [&](int64_t tile, K(&kr)[IPT], uint32_t(&vr)[IPT], bool keys = true, bool vals = !SR) {
    const int64_t base = tile * TILE;
    const K *ks = kin + base + w * WSEG + lane;
    const uint32_t *vs = HAS_V ? vin + base + w * WSEG + lane : nullptr;
    if (base + TILE <= n) {
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        if (keys) kr[i] = ks[i * kWave];
        if constexpr (HAS_V)
          if (vals) vr[i] = vs[i * kWave];
      }
    } else {
      const int valid = static_cast<int>(n - base) - (w * WSEG + lane);
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        if (keys) kr[i] = i * kWave < valid ? ks[i * kWave] : ~K(0);  // pad: max digit, ranked after every real key
        if constexpr (HAS_V)
          if (vals) vr[i] = i * kWave < valid ? vs[i * kWave] : 0u;
      }
    }
  };
  if (PF && first < last) load_tile(first, key, val);
  for (int64_t tile = first; tile < last; ++tile) {
    const int64_t base = tile * TILE;
    const bool full = base + TILE <= n;
#pragma unroll
    for (int k = 0; k < 4; ++k) wcnt[w][lane + kWave * k] = 0;
    // PF: next sub-tile in flight under this one's rank / reorder / scatter;
    // else this sub-tile is loaded here (other workgroups hide the wait)
    K nkey[IPT];
    uint32_t nval[IPT];
    if constexpr (PF) {
      if (tile + 1 < last) load_tile(tile + 1, nkey, nval);
    } else {
      load_tile(tile, key, val);
    }
    // ranks inside the sub-tile (< 65536) two per register
    uint32_t loc[(IPT + 1) / 2];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint32_t d = digit_of(key[i], shift, mask);
      const uint64_t peers = match_any8(d);
      // peers in lanes below mine: mbcnt against the hardware lane mask (no
      // per-lane mask register)
      const uint32_t nbelow = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(peers >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(peers), 0u));
      const uint32_t before = wcnt[w][d];
      const uint32_t r = before + nbelow;
      loc[i / 2] = i & 1 ? loc[i / 2] | r << 16 : r;
      if (nbelow == 0) wcnt[w][d] = before + static_cast<uint32_t>(__popcll(peers));
    }
    __syncthreads();
    // per digit t: wave prefix + sub-tile start into the wave counters, and
    // global base − sub-tile start into gofs
    // (the NW wave counts are read again after the scan instead of being
    // held across it: 16 registers at NW = 16)
    uint32_t tot = 0;
    if (own) {
#pragma unroll
      for (int j = 0; j < NW; ++j) tot += wcnt[j][t];
    }
    uint32_t all;
#ifndef LHPC_SORT_SCAN_TRAIL  // A/B builds: 1 keeps the closing barrier
#define LHPC_SORT_SCAN_TRAIL 0
#endif
    // (the next write of tmp is the next sub-tile's scan, behind its rank
    // barrier; the barrier after the fold below orders this scan's reads.
    // Same box, two runs each: 78.75 / 78.89 G keys/s without the closing
    // barrier, 78.89 / 78.87 with it)
    const uint32_t ts = block_exscan<NW, LHPC_SORT_SCAN_TRAIL != 0>(tot, tmp, all);
    if (own) {
      uint32_t run = ts;
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const uint32_t cj = wcnt[j][t];
        wcnt[j][t] = run;
        run += cj;
      }
      gofs[t] = gb - ts;
      gb += tot;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint32_t p = wcnt[w][digit_of(key[i], shift, mask)] + (i & 1 ? loc[i / 2] >> 16 : loc[i / 2] & 0xFFFFu);
      sk[p] = key[i];
      if constexpr (HAS_V && !SR) sv[p] = val[i];
      if constexpr (SR) {
        loc[i / 2] = i & 1 ? (loc[i / 2] & 0xFFFFu) | p << 16 : (loc[i / 2] & 0xFFFF0000u) | p;
        dg[p] = static_cast<uint8_t>(digit_of(key[i], shift, mask));
      }
    }
    __syncthreads();
    // (no barrier after the scatter: the next sub-tile writes sk, the wcnt
    // columns and gofs only after its rank barrier, which every thread
    // passes once its scatter is done; each wave clears only its own counter
    // row, which only it reads before that barrier)
    const int valid = full ? TILE : static_cast<int>(n - base);
    if constexpr (SR) {
#pragma unroll 8
      for (int k = 0; k < IPT; ++k) {
        const int p = t + BT * k;
        if (full || p < valid) kout[gofs[dg[p]] + static_cast<uint32_t>(p)] = sk[p];
      }
      load_tile(tile, key, val, false, true);  // (L2 hits: under the barrier)
      __syncthreads();  // every key is out of sk: the values take its place
      uint32_t *svr = reinterpret_cast<uint32_t *>(sk);
#pragma unroll
      for (int i = 0; i < IPT; ++i) svr[i & 1 ? loc[i / 2] >> 16 : loc[i / 2] & 0xFFFFu] = val[i];
      __syncthreads();
#pragma unroll 8
      for (int k = 0; k < IPT; ++k) {
        const int p = t + BT * k;
        if (full || p < valid) vout[gofs[dg[p]] + static_cast<uint32_t>(p)] = svr[p];
      }
      continue;
    }
#pragma unroll 8  // (a full unroll holds IPT 64-bit store addresses)
    for (int k = 0; k < IPT; ++k) {
      const int p = t + BT * k;
      if (full || p < valid) {
        const K kk = sk[p];
        const uint32_t g = gofs[digit_of(kk, shift, mask)] + static_cast<uint32_t>(p);
#if defined(LHPC_SORT_PROBE) && LHPC_SORT_PROBE == 1
        // timing-only probe (wrong results): coalesced stores at the input
        // position instead of the digit-run scatter
        kout[base + p] = kk + static_cast<K>(g & 0u);
#else
        kout[g] = kk;
#endif
        if constexpr (HAS_V) vout[g] = sv[p];
      }
    }
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        key[i] = nkey[i];
        if constexpr (HAS_V) val[i] = nval[i];
      }
    }
  }
}

struct DevBuf {
  void *p = nullptr;
  hipStream_t s = nullptr;
  ~DevBuf() {
    if (p) (void)hipFreeAsync(p, s);
  }
  hipError_t alloc(size_t bytes, hipStream_t st) {
    s = st;
    return scratch_alloc(&p, bytes, st);  // library pool (lhpc_common.hpp)
  }
};

// Staging buffers of the host-buffer entry points: plain hipMalloc (not the
// stream-ordered pool) and synchronous copies.  Asynchronous pageable copies
// into pool memory on the null stream were seen to land after the kernel
// that read them (rows read as 0 in 4 of 25 runs of tests/cpp
// test_sparse_grid gpu, the 4-entry Matrix Market case).  Every step of that
// path was ordered on the one caller stream; DESIGN.md §9 traces it and
// records what was ruled out.
struct HostStage {
  void *p = nullptr;
  ~HostStage() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 16); }
};

// resident downsweep blocks on the current device (CUs × blocks per CU),
// cached per kernel and device (relaxed atomics: racing threads compute the
// same value)
template <typename K, bool HAS_V, int IPT, bool PF, int BT, bool SR>
int64_t sort_grid_cap() {
  static std::atomic<int64_t> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return kSortMaxResident;
  std::atomic<int64_t> *slot = dev >= 0 && dev < 64 ? &cache[dev] : nullptr;
  if (slot) {
    const int64_t c = slot->load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_radix_downsweep<K, HAS_V, IPT, PF, BT, SR>, BT, 0) !=
          hipSuccess ||
      cus <= 0 || per_cu <= 0)
    return kSortMaxResident;
  const int64_t cap = std::min<int64_t>(kSortMaxResident, int64_t{cus} * per_cu);
  if (slot) slot->store(cap, std::memory_order_relaxed);
  return cap;
}

template <typename K, bool HAS_V, int IPT, bool PF = true, int BT = kSortThreads, bool SR = false>
int radix_sort_dev(K *keys, uint32_t *vals, int64_t n, int begin_bit, int end_bit, hipStream_t s) {
  if (n <= 1 || begin_bit >= end_bit) return LHPC_OK;
  constexpr int TILE = IPT * BT;
  const int64_t ntiles = (n + TILE - 1) / TILE;
  // Grid: up to 8 waves of resident blocks, but at least ~3 tiles per block. More, shorter blocks even out
  // the tail of the even-share split (500M keys: 768 blocks 8.94 ms, 6144 blocks 8.16 ms); below ~3 tiles
  // per block the per-block digit-count rows outweigh the gain (100M keys: 8192 blocks 1.89 ms, 30000 2.19).
  const int64_t res = sort_grid_cap<K, HAS_V, IPT, PF, BT, SR>();
  // grid sweep knobs of the tuning build only (tools/explore_sort.py; lhpc_common.hpp tuning_env)
  // (1024-thread downsweeps hold one block per CU: twice the waves, the same
  // block count as two 256-thread blocks per CU at 8; 500M keys, same box:
  // 74.3 / 74.9 / 75.0 G keys/s at 4 / 8 / 16)
  constexpr int kWavesDefault = BT >= 1024 ? 16 : 8;
  static const int64_t waves =
      tuning_env("LHPC_SORT_WAVES") ? std::max(1, std::atoi(tuning_env("LHPC_SORT_WAVES"))) : kWavesDefault;
  int64_t cap = std::min<int64_t>(waves * res, std::max<int64_t>(res, ntiles / 3));
  if (const char *e = tuning_env("LHPC_SORT_BLOCKS")) cap = std::max<int64_t>(1, std::atoll(e));
  int64_t nb = std::min<int64_t>(cap, ntiles);
  const int64_t per = (ntiles + nb - 1) / nb;
  nb = (ntiles + per - 1) / per;
  DevBuf k2, v2, counts, dbase;
  LHPC_HIP_TRY(k2.alloc(static_cast<size_t>(n) * sizeof(K), s));
  if (HAS_V) LHPC_HIP_TRY(v2.alloc(static_cast<size_t>(n) * 4, s));
  LHPC_HIP_TRY(counts.alloc(static_cast<size_t>(nb) * 256 * 4, s));
  LHPC_HIP_TRY(dbase.alloc(256 * 4, s));
  K *kin = keys, *kout = static_cast<K *>(k2.p);
  uint32_t *vin = vals, *vout = static_cast<uint32_t *>(v2.p);
  uint32_t *cnt = static_cast<uint32_t *>(counts.p), *db = static_cast<uint32_t *>(dbase.p);
  int passes = 0;
  for (int shift = begin_bit; shift < end_bit; shift += 8, ++passes) {
    const int bits = std::min(8, end_bit - shift);
    const uint32_t mask = (1u << bits) - 1u;
    const int vec16 = (reinterpret_cast<uintptr_t>(kin) & 15u) == 0 ? 1 : 0;
    hipLaunchKernelGGL((k_radix_upsweep<K, TILE>), dim3(static_cast<unsigned>(nb)), dim3(kSortThreads), 0, s, kin,
                       n, shift, mask, per, cnt, vec16);
    hipLaunchKernelGGL(k_radix_scan, dim3(256), dim3(kSortThreads), 0, s, cnt, static_cast<int>(nb), db);
    hipLaunchKernelGGL((k_radix_downsweep<K, HAS_V, IPT, PF, BT, SR>), dim3(static_cast<unsigned>(nb)), dim3(BT), 0,
                       s, kin, kout, vin, vout, n, shift, mask, per, cnt, db);
    std::swap(kin, kout);
    if (HAS_V) std::swap(vin, vout);
  }
  if (passes & 1) {  // result sits in the scratch buffers
    LHPC_HIP_TRY(hipMemcpyAsync(keys, kin, static_cast<size_t>(n) * sizeof(K), hipMemcpyDeviceToDevice, s));
    if (HAS_V) LHPC_HIP_TRY(hipMemcpyAsync(vals, vin, static_cast<size_t>(n) * 4, hipMemcpyDeviceToDevice, s));
  }
  return check_launch(s);
}

// ---------------------------------------------------------------- tile-sum scan
// per-tile sums → exclusive prefix in place (one workgroup), total to *grand
// (16 consecutive sums per thread and step: 150M-entry COO → CSR, 36.6K
// tiles, 81 → 38 µs against one per thread)
__global__ __launch_bounds__(kSortThreads) void k_scan_sums(uint32_t *__restrict__ sums, int64_t nb,
                                                            uint32_t *__restrict__ grand) {
  __shared__ uint32_t tmp[256];
  constexpr int E = 16;
  uint32_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += kSortThreads * E) {
    uint32_t c[E], s = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int64_t i = b0 + threadIdx.x * E + j;
      c[j] = i < nb ? sums[i] : 0u;
      s += c[j];
    }
    uint32_t total;
    uint32_t run = carry + block_exscan256(s, tmp, total);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int64_t i = b0 + threadIdx.x * E + j;
      if (i < nb) sums[i] = run;
      run += c[j];
    }
    carry += total;
  }
  if (threadIdx.x == 0 && grand) *grand = carry;
}

// ---------------------------------------------------------------- COO → CSR
// key = row << col_bits | col; payload = the f32 value's bits (carried through the sort, so no
// permutation gather) or, for f64 values, the input index.
// VEC (rows, cols and values 16-B aligned): four entries per thread, 16-B
// loads and stores (150M entries: 817 → 611 µs against one entry per thread)
template <bool PAY_BITS, bool VEC>
__global__ void k_coo_keys(const int32_t *__restrict__ rows, const int32_t *__restrict__ cols,
                           const uint32_t *__restrict__ vbits, int64_t nnz, int64_t n_rows, int64_t n_cols,
                           int col_bits, uint64_t *__restrict__ keys, uint32_t *__restrict__ pay,
                           int *__restrict__ bad) {
  auto key_of = [&](int32_t r, int32_t c) -> uint64_t {
    if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) {
      atomicOr(bad, 1);
      return 0;
    }
    return (static_cast<uint64_t>(r) << col_bits) | static_cast<uint64_t>(c);
  };
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if constexpr (VEC) {
    typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    const int64_t i = 4 * t;
    if (i + 4 <= nnz) {
      const i32x4 r = __builtin_nontemporal_load(reinterpret_cast<const i32x4 *>(rows) + t);
      const i32x4 c = __builtin_nontemporal_load(reinterpret_cast<const i32x4 *>(cols) + t);
      u64x2 k0 = {key_of(r.x, c.x), key_of(r.y, c.y)}, k1 = {key_of(r.z, c.z), key_of(r.w, c.w)};
      reinterpret_cast<u64x2 *>(keys)[2 * t] = k0;
      reinterpret_cast<u64x2 *>(keys)[2 * t + 1] = k1;
      u32x4 pv;
      if constexpr (PAY_BITS) pv = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(vbits) + t);
      else pv = u32x4{static_cast<uint32_t>(i), static_cast<uint32_t>(i + 1), static_cast<uint32_t>(i + 2),
                      static_cast<uint32_t>(i + 3)};
      reinterpret_cast<u32x4 *>(pay)[t] = pv;
    } else {
      for (int64_t j = i; j < nnz; ++j) {
        keys[j] = key_of(rows[j], cols[j]);
        pay[j] = PAY_BITS ? vbits[j] : static_cast<uint32_t>(j);
      }
    }
  } else {
    if (t >= nnz) return;
    keys[t] = key_of(rows[t], cols[t]);
    pay[t] = PAY_BITS ? vbits[t] : static_cast<uint32_t>(t);
  }
}

// Fused merge (round 6): after the sort, one pass counts the run heads per
// 4096-entry tile (head = key differs from the previous entry's), the tile
// counts are scanned, and one pass per tile recomputes its heads, gives each
// its merged position, sums its run in input order, writes col / val and
// fills the row_ptr entries of the rows that start there — instead of
// heads → scan (reduce, apply) → emit → row_ptr as five passes over the keys.
// Entries are striped over the block (entry b0 + e·256 + t, every load
// coalesced); a head's position within its 64-entry wave row is an mbcnt of
// the row's head ballot, the 64 row counts of the tile are scanned in LDS.
constexpr int kCooTile = 4096;  // 16 rows of 256 entries
constexpr int kCooE = kCooTile / kSortThreads;

__global__ __launch_bounds__(kSortThreads) void k_coo_count(const uint64_t *__restrict__ keys, int64_t nnz,
                                                            uint32_t *__restrict__ sums) {
  __shared__ uint32_t tmp[256];
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kCooTile;
  uint32_t c = 0;
#pragma unroll
  for (int e = 0; e < kCooE; ++e) {
    const int64_t i = b0 + e * kSortThreads + threadIdx.x;
    if (i < nnz) c += (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
  }
  uint32_t total;
  (void)block_exscan256(c, tmp, total);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

template <typename T, bool PAY_BITS, typename O>
__global__ __launch_bounds__(kSortThreads) void k_coo_finish(const uint64_t *__restrict__ keys,
                                                             const uint32_t *__restrict__ pay, int64_t nnz,
                                                             int64_t n_rows, int col_bits,
                                                             const uint32_t *__restrict__ sums,
                                                             const uint32_t *__restrict__ grand, const T *__restrict__ vals,
                                                             int32_t *__restrict__ col_out, T *__restrict__ val_out,
                                                             O *__restrict__ row_ptr) {
  __shared__ uint32_t rc[kCooE * 4];  // head count of each 64-entry wave row, then its exclusive prefix
  auto value = [&](int64_t j) -> T {
    if constexpr (PAY_BITS) return __builtin_bit_cast(T, pay[j]);
    else return vals[pay[j]];
  };
  const int t = threadIdx.x, w = t / kWave, lane = t & (kWave - 1);
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kCooTile;
  uint64_t k[kCooE];
  uint32_t hm = 0, mb[kCooE / 4] = {};  // head bits; the mbcnt of each row, one byte per row
#pragma unroll
  for (int e = 0; e < kCooE; ++e) {
    const int64_t i = b0 + e * kSortThreads + t;
    const bool ok = i < nnz;
    k[e] = ok ? keys[i] : 0;
    const bool h = ok && (i == 0 || k[e] != keys[i - 1]);
    const uint64_t bal = __ballot(h);
    const uint32_t m = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bal >> 32),
                                                 __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bal), 0u));
    mb[e / 4] |= m << (8 * (e % 4));
    hm |= (h ? 1u : 0u) << e;
    if (lane == 0) rc[e * 4 + w] = static_cast<uint32_t>(__popcll(bal));
  }
  __syncthreads();
  if (w == 0) {  // the 64 row counts in entry order (row e, wave w) → exclusive prefix
    const uint32_t v = rc[lane];
    const uint32_t inc = static_cast<uint32_t>(wave_incl_scan(static_cast<int>(v)));
    rc[lane] = inc - v;
  }
  __syncthreads();
  const uint32_t base = sums[blockIdx.x];
  const uint64_t cmask = (uint64_t{1} << col_bits) - 1;
#pragma unroll
  for (int e = 0; e < kCooE; ++e) {
    const int64_t i = b0 + e * kSortThreads + t;
    if (i >= nnz) break;
    if (hm >> e & 1u) {
      const uint32_t pos = base + rc[e * 4 + w] + (mb[e / 4] >> (8 * (e % 4)) & 0xFFu);
      T sv = value(i);
      for (int64_t j = i + 1; j < nnz && keys[j] == k[e]; ++j) sv = sv + value(j);
      col_out[pos] = static_cast<int32_t>(k[e] & cmask);
      val_out[pos] = sv;
      // rows (previous entry's row, this row] start at this merged entry
      const int64_t row = static_cast<int64_t>(k[e] >> col_bits);
      const int64_t prow = i > 0 ? static_cast<int64_t>(keys[i - 1] >> col_bits) : -1;
      for (int64_t r = prow + 1; r <= row; ++r) row_ptr[r] = static_cast<O>(pos);
    }
    if (i == nnz - 1) {  // the rows after the last entry's
      const O g = static_cast<O>(*grand);
      for (int64_t r = static_cast<int64_t>(k[e] >> col_bits) + 1; r <= n_rows; ++r) row_ptr[r] = g;
    }
  }
}

int bits_for(int64_t v) {  // bits to hold values in [0, v)
  int b = 0;
  while (b < 62 && (int64_t{1} << b) < v) ++b;
  return b;
}

template <typename T>
int coo_to_csr_dev(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t *rows, const int32_t *cols,
                   const T *vals, void *row_ptr, int row_ptr_bits, int32_t *col_out, T *val_out,
                   int64_t *nnz_out, hipStream_t s) {
  const int cb = std::max(1, bits_for(n_cols)), rb = std::max(1, bits_for(n_rows));
  if (cb + rb > 64) return LHPC_ERR_UNSUPPORTED;
  const int64_t nt = (nnz + kCooTile - 1) / kCooTile;  // merge tiles
  DevBuf keys, idx, tsum, flag, grand;
  LHPC_HIP_TRY(keys.alloc(static_cast<size_t>(nnz) * 8, s));
  LHPC_HIP_TRY(idx.alloc(static_cast<size_t>(nnz) * 4, s));
  LHPC_HIP_TRY(tsum.alloc(static_cast<size_t>(std::max<int64_t>(nt, 1)) * 4, s));
  LHPC_HIP_TRY(flag.alloc(8, s));
  LHPC_HIP_TRY(grand.alloc(8, s));
  uint64_t *kp = static_cast<uint64_t *>(keys.p);
  uint32_t *ip = static_cast<uint32_t *>(idx.p), *tp = static_cast<uint32_t *>(tsum.p);
  int *bad = static_cast<int *>(flag.p);
  uint32_t *gp = static_cast<uint32_t *>(grand.p);
  LHPC_HIP_TRY(hipMemsetAsync(bad, 0, 8, s));
  LHPC_HIP_TRY(hipMemsetAsync(gp, 0, 8, s));
  const unsigned g = static_cast<unsigned>((std::max<int64_t>(nnz, 1) + 255) / 256);
  constexpr bool kBits = sizeof(T) == 4;
  if (nnz > 0) {
    const bool vec = ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(cols) |
                       (kBits ? reinterpret_cast<uintptr_t>(vals) : 0)) & 15u) == 0;
    if (vec)
      hipLaunchKernelGGL((k_coo_keys<kBits, true>), dim3(static_cast<unsigned>((nnz + 1023) / 1024)), dim3(256), 0,
                         s, rows, cols, reinterpret_cast<const uint32_t *>(vals), nnz, n_rows, n_cols, cb, kp, ip, bad);
    else
      hipLaunchKernelGGL((k_coo_keys<kBits, false>), dim3(g), dim3(256), 0, s, rows, cols,
                         reinterpret_cast<const uint32_t *>(vals), nnz, n_rows, n_cols, cb, kp, ip, bad);
#ifdef LHPC_SORT_P64_VARIANT  // A/B builds
    LHPC_TRY((radix_sort_dev<uint64_t, true, LHPC_SORT_P64_VARIANT>(kp, ip, nnz, 0, cb + rb, s)));
#else
    LHPC_TRY((radix_sort_dev<uint64_t, true, 16, false, 1024, true>(kp, ip, nnz, 0, cb + rb, s)));
#endif
    const dim3 tg(static_cast<unsigned>(nt));
    hipLaunchKernelGGL(k_coo_count, tg, dim3(kSortThreads), 0, s, kp, nnz, tp);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kSortThreads), 0, s, tp, nt, gp);
    if (row_ptr_bits == 64)
      hipLaunchKernelGGL((k_coo_finish<T, kBits, int64_t>), tg, dim3(kSortThreads), 0, s, kp, ip, nnz, n_rows, cb, tp,
                         gp, vals, col_out, val_out, static_cast<int64_t *>(row_ptr));
    else
      hipLaunchKernelGGL((k_coo_finish<T, kBits, int32_t>), tg, dim3(kSortThreads), 0, s, kp, ip, nnz, n_rows, cb, tp,
                         gp, vals, col_out, val_out, static_cast<int32_t *>(row_ptr));
  } else {  // no entries: row_ptr all zeros
    LHPC_HIP_TRY(hipMemsetAsync(row_ptr, 0, static_cast<size_t>(n_rows + 1) * (row_ptr_bits / 8), s));
  }
  LHPC_TRY(check_launch(s));
  // the two status words are read after the stream has drained, with
  // synchronous copies: no asynchronous copy touches pageable host memory
  // anywhere in the COO->CSR path
  int hbad = 0;
  uint32_t hnnz = 0;
  LHPC_HIP_TRY(hipStreamSynchronize(s));
  LHPC_HIP_TRY(hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost));
  LHPC_HIP_TRY(hipMemcpy(&hnnz, gp, 4, hipMemcpyDeviceToHost));
  if (hbad) return LHPC_ERR_INVALID_ARG;
  if (nnz_out) *nnz_out = hnnz;
  return LHPC_OK;
}

}  // namespace
}  // namespace lhpc

using namespace lhpc;

namespace {
template <typename K, bool HAS_V, int IPT, bool PF = true, int BT = kSortThreads, bool SR = false>
int sort_entry(K *keys, uint32_t *vals, int64_t n, int begin_bit, int end_bit, int on_device, void *stream) {
  constexpr int KB = static_cast<int>(sizeof(K) * 8);
  if (n < 0 || (!keys && n > 0) || (HAS_V && !vals && n > 0) || begin_bit < 0 || end_bit > KB ||
      begin_bit > end_bit)
    return LHPC_ERR_INVALID_ARG;
  if (n >= (int64_t{1} << 32)) return LHPC_ERR_UNSUPPORTED;  // 32-bit ranks
  RocTxRange rx("lhpc_radix_sort");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (on_device) return radix_sort_dev<K, HAS_V, IPT, PF, BT, SR>(keys, vals, n, begin_bit, end_bit, s);
  HostStage dk, dv;
  LHPC_HIP_TRY(dk.alloc(static_cast<size_t>(n) * sizeof(K)));
  if (HAS_V) LHPC_HIP_TRY(dv.alloc(static_cast<size_t>(n) * 4));
  LHPC_HIP_TRY(hipMemcpy(dk.p, keys, static_cast<size_t>(n) * sizeof(K), hipMemcpyHostToDevice));
  if (HAS_V) LHPC_HIP_TRY(hipMemcpy(dv.p, vals, static_cast<size_t>(n) * 4, hipMemcpyHostToDevice));
  LHPC_TRY((radix_sort_dev<K, HAS_V, IPT, PF, BT, SR>(static_cast<K *>(dk.p), static_cast<uint32_t *>(dv.p), n, begin_bit,
                                          end_bit, s)));
  LHPC_HIP_TRY(hipStreamSynchronize(s));
  LHPC_HIP_TRY(hipMemcpy(keys, dk.p, static_cast<size_t>(n) * sizeof(K), hipMemcpyDeviceToHost));
  if (HAS_V) LHPC_HIP_TRY(hipMemcpy(vals, dv.p, static_cast<size_t>(n) * 4, hipMemcpyDeviceToHost));
  return LHPC_OK;
}
}  // namespace

// Round 6 (profiles/r06/ab_sort2): 1024-thread blocks without the prefetch,
// one block per CU at 4 waves per SIMD (≤ 128 VGPRs) — twice the waves of
// the 256-thread 8192-key kernel (246 VGPRs, 2 per SIMD) and longer digit
// runs.  Keys only: 20480-key sub-tiles with the next sub-tile's keys
// prefetched into registers (20 + 20 keys per thread, 127 VGPRs once the
// lanes-below count is an mbcnt), 500M keys 65.9 → 75.0 (16384, no
// prefetch) → 78.6 (24576, no prefetch; 28 / 32 keys spill) → 81.1 G keys/s;
// 12288 keys 70.7; 16384 as 512 × 32 at 2 per SIMD 68.7; 12288 as 512 × 24,
// two blocks per CU, 71.3.  32-bit pairs:
// 16384 (values in their own LDS array), 150M pairs 4.17 → 3.53 ms.  64-bit
// pairs: 16384 with the split reorder (SR: keys, then values, through one
// 128 KB buffer; 127 VGPRs), 150M pairs over 47 bits 8.70 → 7.77 ms, COO→CSR
// 12.0 → 11.8 ms; 12288 with SR 8.07; 8192 as 1024 × 8 8.75 (no gain).
// Round 3: 8192-key sub-tiles (32 keys per thread, 246 VGPRs, 2 waves per
// SIMD): digit runs twice as long, so the scatter writes whole 128-B lines,
// and half the per-sub-tile scans and barriers per key — same box, three runs
// each, 500M keys 8.92 → 7.68 ms against 4096-key sub-tiles (16384-key
// sub-tiles without the prefetch: 406 VGPRs, 10.15 ms).  64-bit pairs (the
// COO→CSR sort): 8192-key sub-tiles without the next-sub-tile prefetch (288
// VGPRs): 150M pairs over 47 bits 8.29 → 7.61 ms, COO→CSR 12.66 → 11.72 ms;
// 32-bit pairs the same way: 150M pairs 4.67 → 4.00 ms.  (Keys only, same
// box: 6144-key sub-tiles 8.24 ms and 8192 without the prefetch 7.33 ms,
// against 7.19 ms.)
extern "C" int lhpc_radix_sort_u32(uint32_t *keys, int64_t n, int begin_bit, int end_bit, int on_device,
                                   void *stream) {
  try {
#ifdef LHPC_SORT_KEYS_VARIANT  // A/B builds: IPT, PF, BT of the keys-only downsweep
    return sort_entry<uint32_t, false, LHPC_SORT_KEYS_VARIANT>(keys, nullptr, n, begin_bit, end_bit, on_device, stream);
#else
    return sort_entry<uint32_t, false, 20, true, 1024>(keys, nullptr, n, begin_bit, end_bit, on_device, stream);
#endif
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_radix_sort_pairs_u32(uint32_t *keys, uint32_t *vals, int64_t n, int begin_bit, int end_bit,
                                         int on_device, void *stream) {
  try {
#ifdef LHPC_SORT_P32_VARIANT  // A/B builds
    return sort_entry<uint32_t, true, LHPC_SORT_P32_VARIANT>(keys, vals, n, begin_bit, end_bit, on_device, stream);
#else
    return sort_entry<uint32_t, true, 16, false, 1024>(keys, vals, n, begin_bit, end_bit, on_device, stream);
#endif
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_radix_sort_pairs_u64(uint64_t *keys, uint32_t *vals, int64_t n, int begin_bit, int end_bit,
                                         int on_device, void *stream) {
  try {
#ifdef LHPC_SORT_P64_VARIANT  // A/B builds
    return sort_entry<uint64_t, true, LHPC_SORT_P64_VARIANT>(keys, vals, n, begin_bit, end_bit, on_device, stream);
#else
    return sort_entry<uint64_t, true, 16, false, 1024, true>(keys, vals, n, begin_bit, end_bit, on_device, stream);
#endif
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_coo_to_csr(int dtype, int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t *rows,
                               const int32_t *cols, const void *vals, void *row_ptr, int row_ptr_bits,
                               int32_t *col_out, void *val_out, int64_t *nnz_out, int on_device, void *stream) {
  try {
    if (n_rows < 0 || n_cols < 0 || nnz < 0 || !row_ptr || (row_ptr_bits != 32 && row_ptr_bits != 64) ||
        (nnz > 0 && (!rows || !cols || !vals || !col_out || !val_out)) || (dtype != LHPC_F32 && dtype != LHPC_F64))
      return LHPC_ERR_INVALID_ARG;
    if (nnz >= (int64_t{1} << 32) || (row_ptr_bits == 32 && nnz >= (int64_t{1} << 31))) return LHPC_ERR_UNSUPPORTED;
    RocTxRange rx("lhpc_coo_to_csr");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t vb = dtype == LHPC_F32 ? 4 : 8;
    auto run = [&](const int32_t *r, const int32_t *c, const void *v, void *rp, int32_t *co, void *vo,
                   int64_t *un) -> int {
      if (dtype == LHPC_F32)
        return coo_to_csr_dev<float>(n_rows, n_cols, nnz, r, c, static_cast<const float *>(v), rp, row_ptr_bits, co,
                                     static_cast<float *>(vo), un, s);
      return coo_to_csr_dev<double>(n_rows, n_cols, nnz, r, c, static_cast<const double *>(v), rp, row_ptr_bits, co,
                                    static_cast<double *>(vo), un, s);
    };
    if (on_device) return run(rows, cols, vals, row_ptr, col_out, val_out, nnz_out);
    const size_t rpb = static_cast<size_t>(n_rows + 1) * (row_ptr_bits / 8);
    HostStage dr, dc, dv, drp, dco, dvo;
    LHPC_HIP_TRY(dr.alloc(static_cast<size_t>(nnz) * 4));
    LHPC_HIP_TRY(dc.alloc(static_cast<size_t>(nnz) * 4));
    LHPC_HIP_TRY(dv.alloc(static_cast<size_t>(nnz) * vb));
    LHPC_HIP_TRY(drp.alloc(rpb));
    LHPC_HIP_TRY(dco.alloc(static_cast<size_t>(nnz) * 4));
    LHPC_HIP_TRY(dvo.alloc(static_cast<size_t>(nnz) * vb));
    if (nnz > 0) {
      LHPC_HIP_TRY(hipMemcpy(dr.p, rows, static_cast<size_t>(nnz) * 4, hipMemcpyHostToDevice));
      LHPC_HIP_TRY(hipMemcpy(dc.p, cols, static_cast<size_t>(nnz) * 4, hipMemcpyHostToDevice));
      LHPC_HIP_TRY(hipMemcpy(dv.p, vals, static_cast<size_t>(nnz) * vb, hipMemcpyHostToDevice));
    }
    int64_t un = 0;
    LHPC_TRY(run(static_cast<int32_t *>(dr.p), static_cast<int32_t *>(dc.p), dv.p, drp.p,
                 static_cast<int32_t *>(dco.p), dvo.p, &un));  // ends with a stream synchronize
    LHPC_HIP_TRY(hipMemcpy(row_ptr, drp.p, rpb, hipMemcpyDeviceToHost));
    if (un > 0) {
      LHPC_HIP_TRY(hipMemcpy(col_out, dco.p, static_cast<size_t>(un) * 4, hipMemcpyDeviceToHost));
      LHPC_HIP_TRY(hipMemcpy(val_out, dvo.p, static_cast<size_t>(un) * vb, hipMemcpyDeviceToHost));
    }
    if (nnz_out) *nnz_out = un;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}
