/*
 * lhpc.h — C ABI of the MI355X-native libHPC hot path (CSR SpMV + ghost-cell
 * stencils).  Every entry point is `extern "C"`, takes plain pointers and
 * sizes, and returns an `int` status:
 *
 *     0              success (LHPC_OK)
 *     < 0            lhpc error (see lhpc_status below)
 *     > 0            a wrapped hipError_t value, or LHPC_RCCL_STATUS_BASE +
 *                    ncclResult_t for a failed RCCL call (lhpc_dist_*)
 *
 * No exception crosses this boundary.  The C++ drop-in headers
 * (include/hpc/ and include/sparse/ headers) map a non-zero status to
 * std::system_error, mirroring the reference's cudahelper::throwCudaError
 * convention (reference lib/gpu/util/include/cudaHelper.cuh:10-27).
 *
 * What each entry point replaces in the reference
 * ------------------------------------------------
 * The reference (Liupeter01/libHPC) has NO CSR SpMV anywhere:
 * the SpMV entry points below are a new operator in the reference's
 * `sparse` namespace idiom (lib/sparse/include/RootGrid.hpp:10-22 is the
 * existing `sparse::` API), fed by the reference's host layout contract
 * hpc::HPCHighDimensionFlatArray<1,T> (lib/hpc/include/HPCHighDimensionFlatArray.hpp:54-57).
 *
 * The stencil entry points replace the 17-tap box blurs of
 * tests/test_hpc_benchmark/test_hpc_benchmark.cpp:354-368 (x) and :444-457 (y)
 * and their SSE twins :425-441 / :575-601, operating on the same padded
 * row-major buffers hpc::HPCHighDimensionFlatArray<2,float,nblur> (input, `a`
 * at :32) and <2,float> (output, `b` at :33).
 *
 * Threading: a plan is not thread-safe; drive it from one host thread.
 * All compute calls are asynchronous on the given stream (`void*` is a
 * hipStream_t; NULL = the null stream) unless a host pointer is passed, in
 * which case the call synchronises that stream before returning.
 */
#ifndef LHPC_H_
#define LHPC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LHPC_ABI_VERSION 1

/* ---------------------------------------------------------------- status */
enum lhpc_status {
  LHPC_OK = 0,
  LHPC_ERR_INVALID_ARG = -1,   /* null pointer, negative size, bad enum     */
  LHPC_ERR_BAD_CSR = -2,       /* row_ptr not monotone / col out of range   */
  LHPC_ERR_ALLOC = -3,         /* device or host allocation failed          */
  LHPC_ERR_NO_DEVICE = -4,     /* no usable gfx950 device                   */
  LHPC_ERR_UNSUPPORTED = -5,   /* valid request the build does not support  */
  LHPC_ERR_INTERNAL = -6,
  LHPC_ERR_BUSY = -7           /* plan-owned work already in use (CG solve) */
};
/* RCCL failures: LHPC_RCCL_STATUS_BASE + ncclResult_t (above any hipError_t) */
#define LHPC_RCCL_STATUS_BASE 10000

/* ----------------------------------------------------------------- dtype */
enum lhpc_dtype { LHPC_F32 = 0, LHPC_F64 = 1 };

/* --------------------------------------------------------- plan flags   */
enum lhpc_plan_flags {
  LHPC_PLAN_DEFAULT = 0,
  LHPC_PLAN_VALIDATE = 1u << 0,     /* check row_ptr monotone, cols in range  */
  LHPC_PLAN_DEVICE_INPUT = 1u << 1, /* row_ptr/col_idx/val are device ptrs on the
                                       plan's device: validated there; XTILE
                                       layouts are built on the GPU (others
                                       copy A to the host first)              */
  /* force a kernel family instead of the heuristic (testing / benchmarks)   */
  LHPC_PLAN_FORCE_ROWGROUP = 1u << 4,
  LHPC_PLAN_FORCE_ADAPTIVE = 1u << 5,
  LHPC_PLAN_FORCE_XSLICE = 1u << 6,
  /* XSLICE per-slice partial sums.  Every slice's row sum is accumulated in
   * fp64 registers; the S partials are then summed in fp64 in slice order.
   * Default for fp32 data: partials stored as fp32 (one rounding each), error
   * ≤ 2^-23·Σ|a·x| — 8× inside the 1e-6·Σ|a·x| bar.  EXACT_PARTIALS stores
   * them as fp64 (error 2^-24·|y| + O(2^-50)·Σ|a·x|, ~10% slower at C2).
   * fp64 data always uses fp64 partials.  FAST_PARTIALS is the fp32 default,
   * kept as a flag for callers that name it.                               */
  LHPC_PLAN_FAST_PARTIALS = 1u << 7,
  LHPC_PLAN_EXACT_PARTIALS = 1u << 8,
  LHPC_PLAN_FORCE_XTILE = 1u << 9,
  LHPC_PLAN_FORCE_SELL = 1u << 10  /* LHPC_ERR_UNSUPPORTED past 8 nonzeros per row */
};

/* kernel families a plan can select (lhpc_spmv_plan_info.kernel)          */
enum lhpc_spmv_kernel {
  LHPC_KERNEL_ROWGROUP = 0, /* L lanes per row, wave64 DPP reduction        */
  LHPC_KERNEL_ADAPTIVE = 1, /* nnz-balanced row blocks + long-row split     */
  LHPC_KERNEL_XSLICE = 2,   /* XCD-local column slices + partial reduce     */
  LHPC_KERNEL_XTILE = 3,    /* x tiles in LDS: tile gather + chunk reduce   */
  LHPC_KERNEL_SELL = 4      /* rows ≤ 8 nonzeros: lane per row, 64-row slices */
};

typedef struct lhpc_spmv_plan lhpc_spmv_plan;

typedef struct lhpc_spmv_plan_info {
  int dtype;
  int kernel;          /* enum lhpc_spmv_kernel                             */
  int lanes_per_row;   /* ROWGROUP: L in {4,8,16,32,64}                     */
  int rows_per_group;  /* ROWGROUP: rows per lane group per launch step     */
  int64_t n_rows, n_cols, nnz;
  int64_t n_blocks;    /* ADAPTIVE / SELL: row blocks (SELL: 256 rows each)  */
  int64_t n_long_rows; /* ADAPTIVE: rows split across workgroups            */
  int64_t device_bytes;/* HBM held by the plan                              */
  int device;          /* HIP device ordinal                                */
  int launches;        /* kernel launches per lhpc_spmv call                */
  int slices;          /* XSLICE: column slices S (8 per XCD phase);
                          XTILE: x tiles S                                  */
  int64_t slice_width; /* XSLICE / XTILE: columns per slice / tile          */
} lhpc_spmv_plan_info;

/* ------------------------------------------------------- variant options
 * Kernel-variant and tuning choices, passed explicitly to the *_opts entry
 * points below: the library never reads the process environment, so the
 * same call always builds the same plan.  Every field at 0 means the
 * automatic choice, i.e. exactly what the plain entry points do.  Call
 * lhpc_options_init first; struct_size (set by it) lets later ABI versions
 * append fields.  The reference has no runtime knobs at all (compile-time
 * template parameters only, SURVEY §5 "Config / flags"); these exist for the
 * measured alternatives of DESIGN.md §4 and for tests that pin a variant.
 */
enum lhpc_xtile_reduce {
  LHPC_XTILE_REDUCE_AUTO = 0,
  LHPC_XTILE_REDUCE_PERM = 1,   /* scatter xg into CSR slots through perm     */
  LHPC_XTILE_REDUCE_IPERM = 2   /* gather CSR positions through iperm         */
};
enum lhpc_xtile_align {
  LHPC_XTILE_ALIGN_AUTO = 0,
  LHPC_XTILE_ALIGN_OFF = 1,     /* segments packed back to back               */
  LHPC_XTILE_ALIGN_UNITS = 2    /* every segment padded to 16 B (iperm only)  */
};
enum lhpc_stencil7_impl {
  LHPC_S7_AUTO = 0,
  LHPC_S7_SIMPLE = 1,           /* thread per column                          */
  LHPC_S7_RING = 2,             /* buffer-addressed dword register ring       */
  LHPC_S7_RING_X4 = 3,          /* x4 ring (16-B rows per lane)               */
  LHPC_S7_RING_X4_LDS = 4       /* x4 ring, inner halo rows shared via LDS    */
};
enum lhpc_store_policy {
  LHPC_STORE_AUTO = 0,
  LHPC_STORE_PLAIN = 1,
  LHPC_STORE_NT = 2,            /* non-temporal                               */
  LHPC_STORE_STAGED = 3         /* stencil7 dword ring: float4 via LDS rows   */
};
enum lhpc_dist_exchange {
  LHPC_DIST_EXCHANGE_AUTO = 0,  /* peer stores when y is a registered window, else RCCL */
  LHPC_DIST_EXCHANGE_RCCL = 1,  /* in-place all-gather / broadcast group      */
  LHPC_DIST_EXCHANGE_P2P = 2,   /* direct xGMI peer stores (y must be a window) */
  LHPC_DIST_EXCHANGE_NONE = 3   /* local rows only (SpMV-only timing)         */
};
typedef struct lhpc_options {
  uint32_t struct_size;         /* sizeof(lhpc_options), set by lhpc_options_init */
  /* SpMV kernel selection */
  int32_t spmv_no_xtile;        /* 1: gathers without locality get XSLICE, not XTILE */
  double spmv_locality;         /* distinct x lines per nonzero above which gathers
                                   count as random (0: 0.25)                      */
  int32_t rowgroup_lanes;       /* ROWGROUP: lanes per row L (0: from the mean)  */
  int32_t rowgroup_rows;        /* ROWGROUP: rows per lane group R               */
  /* XTILE */
  int32_t xtile_reduce;         /* enum lhpc_xtile_reduce                        */
  int32_t xtile_ranges;         /* 1: one range; K ≥ 2: K cache-sized row ranges */
  int32_t xtile_steps;          /* gather steps in flight: 2, 4, 8 (auto), 16 (fp32; fp64 caps at 8) */
  int32_t xtile_store;          /* xg stores: LHPC_STORE_PLAIN / _NT             */
  int32_t xtile_cut;            /* chunk-cut window in nonzeros (0: M/32)        */
  int32_t xtile_align;          /* enum lhpc_xtile_align                         */
  int64_t xtile_piece;          /* gather piece length in nonzeros               */
  int64_t xtile_range_piece;    /* the same under cache-sized ranges             */
  /* XSLICE */
  int32_t xslice_slices;        /* column slices S (rounded to a multiple of 8)  */
  int32_t xslice_partial;       /* 1: fp32 partials, 2: fp64 partials            */
  int32_t xslice_window;        /* 64-nonzero windows per chunk pass (1..4)      */
  int32_t xslice_reserved;
  double xslice_mb;             /* target x slice size in MB (0: 5)              */
  /* stencils */
  int32_t stencil7_impl;        /* enum lhpc_stencil7_impl                       */
  int32_t stencil7_store;       /* enum lhpc_store_policy                        */
  int32_t stencil7_ry;          /* ring tile: rows per wave (1, 2, 4)            */
  int32_t stencil7_nj;          /* ring tile: 64-column blocks per wave (4, 8)   */
  int32_t stencil7_zc;          /* z planes per block (0: grid ≈ stencil7_blocks) */
  int32_t stencil7_pf;          /* prefetch planes (1..3)                        */
  int32_t stencil7_blocks;      /* target grid size (0: 256)                     */
  int32_t blur_x_rows;          /* blur_x rows per wave (1, 2, 4, 8, 16, 32)     */
  int32_t blur_y_vec;           /* blur_y columns per thread (1, 2, 4)           */
  int32_t blur_y_rows;          /* blur_y output rows per thread (16 … 64)       */
  /* multi-GPU SpMV (lhpc_dist_spmv) */
  int32_t dist_exchange;        /* enum lhpc_dist_exchange                       */
  int32_t dist_broadcast;       /* 1: RCCL broadcast groups even for equal blocks */
  int32_t dist_world1;          /* 1: issue the RCCL exchange at world 1 (tests) */
  /* XTILE row parts: a matrix whose tile stream does not fit the int32
   * stream offsets (nnz + 8·tiles ≥ 2^31) is cut into nnz-balanced row parts,
   * one XTILE plan each, run in turn on the same x.  0: parts only past that
   * limit; > 0: at most this many nonzeros per part (tests: the split path
   * at small sizes)                                                          */
  int32_t xtile_part_nnz;
  /* single-process multi-device plans (n_devices > 1) */
  int32_t multi_chunks;         /* row chunks per device K (0: 2)                */
  int32_t multi_exchange;       /* enum lhpc_dist_exchange: AUTO/P2P = peer
                                   stores, RCCL = ncclCommInitAll group
                                   all-gathers (distinct devices only)          */
  int32_t multi_force;          /* 1: the multi-device path even for one device */
  int32_t dist_reduce_streams;  /* lhpc_dist_spmv: chunk reduces alternate over this many
                                   streams (1 or 2; 0: 2), so chunk k+1 fills the CUs
                                   chunk k's tail leaves idle                        */
  /* XTILE column blocks: when x spans many tiles (n_cols past ≈ 30M fp32 /
   * 15M fp64) each reduce chunk meets every tile in a few nonzeros, so the
   * plan cuts the columns into B blocks, one XTILE plan each over x's column
   * range, run in turn, every block after the first adding into y.  0: auto,
   * 1: never, B ≥ 2: B blocks (tests: the path at small sizes)               */
  int32_t xtile_col_blocks;
  /* XTILE layout build for host-buffer CSR: 0 (auto) uploads A and builds on
   * the GPU (byte-identical to the host build, several times faster), 1
   * builds on the host (tests compare the two)                              */
  int32_t xtile_host_build;
  /* 1: short rows with x locality stay on ADAPTIVE instead of SELL (rows of
   * ≤ 8 nonzeros whose padded slices stream no more bytes than CSR)        */
  int32_t spmv_no_sell;
  /* XTILE cache-sized ranges (no user splits, iperm reduce): 0 (auto) one
   * range-sized xg ring reused by every range, so a range's gather overwrites
   * lines still in the Infinity Cache instead of evicting dirty ones to HBM;
   * 1: one xg slot per stream entry (the round-5 layout); 2: the ring for
   * user row ranges too (whole calls only; the per-rank plans of
   * lhpc_dist_spmv ask for it).  Ring plans refuse lhpc_spmv_stage /
   * lhpc_spmv_range (LHPC_ERR_UNSUPPORTED).                                 */
  int32_t xtile_ring;
  /* XTILE iperm reduce (≤ 512 fp32 / 1024 fp64 tiles): 1 the segment scan
   * per chunk; 2 the plan's per-chunk phase-A tables (batch rank terms and
   * segment bases, copied to LDS by LDS-DMA); 0 (auto): 2 for fp64, 1 fp32 */
  int32_t xtile_pretable;
} lhpc_options;
void lhpc_options_init(lhpc_options *opts);

/* ------------------------------------------------------------- runtime   */
const char *lhpc_strerror(int status);
int lhpc_abi_version(void);
/* Build tag of this library, bit flags; 0 for the product build.  Loaders
 * (libhpc_amd/__init__.py with LHPC_LIB_PATH) refuse LHPC_BUILD_PROBE, a
 * timing-only build that skips work and computes wrong results.           */
#define LHPC_BUILD_TUNING 1 /* reads LHPC_* tuning variables (tools/ A/B)     */
#define LHPC_BUILD_DEBUG 2  /* device bounds traps, synchronous launch checks */
#define LHPC_BUILD_PROBE 4  /* timing-only probe: wrong results               */
#define LHPC_BUILD_AB 8     /* an A/B variant of the product kernels          */
int lhpc_build_flags(void);
/* number of visible gfx950 devices (0 when none; never an error)          */
int lhpc_device_count(void);

/* ------------------------------------------------------------ CSR SpMV   */
/*
 * Create a plan for y = A·x with A an n_rows × n_cols CSR matrix.
 *   dtype        LHPC_F32 or LHPC_F64 (type of val, x, y)
 *   row_ptr      n_rows+1 offsets, int32 (row_ptr_bits = 32) or int64 (64)
 *   col_idx      nnz int32 column indices in [0, n_cols)
 *   val          nnz values of dtype
 *   device_ids   HIP device ordinals; NULL = current device
 *   n_devices    1: one device.  > 1 (≤ 16): a single-process multi-device
 *                plan: the rows are cut into n_devices·K
 *                nnz-balanced blocks (K = options.multi_chunks, default 2;
 *                block k·n_devices + d is device d's chunk k), each device
 *                gets its own local plan, stream and comm stream (and RCCL
 *                comm with options.multi_exchange = RCCL), peer access is
 *                enabled between the listed devices.  lhpc_spmv then takes x
 *                and y on device_ids[0] (or host buffers): x is copied to the
 *                other devices, every device computes its blocks, the blocks
 *                come back into y.  lhpc_spmv_multi keeps full replicas on
 *                every device instead.  A device may be listed twice (tests:
 *                several "devices" sharing one GPU; peer stores only).  The
 *                alternative, one process per GPU, is lhpc_dist_* below.
 * The plan COPIES A into HBM (and may re-encode it); it never retains the
 * caller's pointers after returning.
 */
int lhpc_spmv_plan_create(lhpc_spmv_plan **out, int dtype, int64_t n_rows,
                          int64_t n_cols, int64_t nnz, const void *row_ptr,
                          int row_ptr_bits, const int32_t *col_idx,
                          const void *val, const int *device_ids,
                          int n_devices, unsigned flags);
/*
 * y = A·x.  With buffers_on_device != 0, x (n_cols) and y (n_rows) are HBM
 * pointers and the call is fully asynchronous on `stream`.  Otherwise they
 * are host pointers: x is staged through a plan-owned HBM buffer, y copied
 * back, and the stream synchronised before return.
 */
int lhpc_spmv(lhpc_spmv_plan *plan, const void *x, void *y,
              int buffers_on_device, void *stream);
int lhpc_spmv_plan_info_get(const lhpc_spmv_plan *plan,
                            lhpc_spmv_plan_info *info);
/* Test support: 64-bit FNV-1a digests (size folded in) of an XTILE plan's
 * device layout arrays — row_ptr, col16, perm/iperm, val runs, chunk
 * descriptors, cr, segment table lo/len and hi, gather pieces, cont — into
 * out[0..9] (cap ≥ 10), *n_out = 10; a plan of row parts / column blocks
 * folds its parts' digests in order.  LHPC_ERR_UNSUPPORTED for other plans.
 * A plan built from LHPC_PLAN_DEVICE_INPUT has the same digests as the host
 * build of the same matrix and options.                                     */
int lhpc_spmv_plan_layout_digest(const lhpc_spmv_plan *plan, uint64_t *out, int cap, int *n_out);
/*
 * Multi-device plans: y = A·x with full replicas on every device.  x[d]
 * (n_cols) and y[d] (n_rows, not x[d]) are HBM pointers on device d; after
 * the call every y[d] holds the whole y (so y is the next x of an iterative
 * loop with no host round trip).  streams[d]: the stream on device d the
 * call is ordered on (NULL array: the plan's own streams); the call is
 * asynchronous on them.  Device d reduces its chunk k into y[d] and its comm
 * stream stores that block into every other y[p] (xGMI peer stores: all
 * links at once) while chunk k+1 is reduced; with options.multi_exchange =
 * RCCL one group of in-place all-gathers per chunk instead.  No other
 * stream may read y[d] until its stream passes the call.  Replaces the
 * per-GPU SpMV calls a single-process caller of the reference would make
 * (SURVEY §8b "Threading"; no reference interface: the reference has no
 * multi-device code).
 */
int lhpc_spmv_multi(lhpc_spmv_plan *plan, const void *const *x, void *const *y, void *const *streams);
/* the split of a plan: devices, chunks K, exchange (enum lhpc_dist_exchange;
 * NONE for a single-device plan), device ordinals (capacity n_devices) and
 * the n_devices·K + 1 row cuts; any output may be NULL.  A single-device plan
 * reports one device, K = 1 and cuts {0, n_rows}.                           */
int lhpc_spmv_plan_multi_info(const lhpc_spmv_plan *plan, int *n_devices, int *chunks, int *exchange,
                              int *device_ids, int64_t *cuts);
/*
 * Row-range plans for overlapping a collective with the SpMV (one process
 * per GPU, libhpc_amd/dist.py): as lhpc_spmv_plan_create, with the plan's
 * work cut at every row in split_rows (ascending, in (0, n_rows)), so that
 * range k = rows [split_rows[k-1], split_rows[k]) (split_rows[-1] = 0,
 * split_rows[n_splits] = n_rows) can be finished on its own:
 *   lhpc_spmv_stage(plan, x, stream)        stages x (the XTILE tile gather)
 *   lhpc_spmv_range(plan, k, y_k, stream)   writes range k's rows to y_k
 * Device buffers only, asynchronous on `stream`; all ranges of one x follow
 * one stage on the same stream.  LHPC_ERR_UNSUPPORTED when the matrix does
 * not select the XTILE layout (gathers with locality, or x ≤ 8 MB): use one
 * plan per range then.  lhpc_spmv on such a plan computes every range; when
 * the plan's gathered x stream exceeds the GPU's Infinity Cache (fp32, > 256
 * MB) it runs gather k then reduce k per range, and lhpc_dist_spmv does the
 * same per chunk (results identical to stage + ranges).
 * Replaces the per-block SpMV calls of the reference's row-block split
 * (no reference interface).
 */
int lhpc_spmv_plan_create_split(lhpc_spmv_plan **out, int dtype, int64_t n_rows,
                                int64_t n_cols, int64_t nnz, const void *row_ptr,
                                int row_ptr_bits, const int32_t *col_idx,
                                const void *val, const int *device_ids,
                                int n_devices, unsigned flags, int n_splits,
                                const int64_t *split_rows);
/* Both of the above with explicit variant options (NULL = all automatic);
 * n_splits = 0 gives an ordinary plan.                                      */
int lhpc_spmv_plan_create_opts(lhpc_spmv_plan **out, int dtype, int64_t n_rows,
                               int64_t n_cols, int64_t nnz, const void *row_ptr,
                               int row_ptr_bits, const int32_t *col_idx,
                               const void *val, const int *device_ids,
                               int n_devices, unsigned flags, int n_splits,
                               const int64_t *split_rows,
                               const lhpc_options *opts);
int lhpc_spmv_stage(const lhpc_spmv_plan *plan, const void *x, void *stream);
int lhpc_spmv_range(const lhpc_spmv_plan *plan, int k, void *y_range, void *stream);
int lhpc_spmv_plan_destroy(lhpc_spmv_plan *plan);

/*
 * nnz-balanced contiguous row split for one-process-per-GPU SpMV:
 * cuts[0] = 0, cuts[parts] = n_rows, and cuts[p] is the smallest row r with
 * row_ptr[r] >= ceil(p·nnz/parts) (binary search on row_ptr).  Host only.
 */
int lhpc_csr_partition_rows(const void *row_ptr, int row_ptr_bits,
                            int64_t n_rows, int parts, int64_t *cuts);

/* -------------------------------------------------------- stencils      */
/*
 * 17-tap (2·nblur+1) box blur along x of a ghost-padded 2-D grid, the
 * reference's BM_x_blur (test_hpc_benchmark.cpp:354-368):
 *     b(y,x) = Σ_{k=-nblur..nblur} a(y, x+k), ascending k, from 0.0f.
 * `a` has layout HPCHighDimensionFlatArray<2,float,ghost>: physical row
 * length nx + 2·ghost, ny + 2·ghost rows; logical (y,x) lives at
 * (y+ghost)·(nx+2·ghost) + (x+ghost).  `b` is HPCHighDimensionFlatArray<2,float,0>
 * (ny × nx, row-major).  Requires ghost >= nblur.
 */
int lhpc_blur_x_f32(const float *a, float *b, int64_t ny, int64_t nx,
                    int64_t ghost, int nblur, int buffers_on_device,
                    void *stream);
/* y-direction twin: b(y,x) = Σ_k a(y+k, x) (test_hpc_benchmark.cpp:444-457) */
int lhpc_blur_y_f32(const float *a, float *b, int64_t ny, int64_t nx,
                    int64_t ghost, int nblur, int buffers_on_device,
                    void *stream);
/*
 * 7-point 3-D stencil on HPCHighDimensionFlatArray<3,float,ghost> buffers
 * (ghost >= 1), both u and out with the same padded layout:
 *   out(z,y,x) = c0·u + c1·(((((u(z-1)+u(z+1)) + u(y-1)) + u(y+1)) + u(x-1)) + u(x+1))
 * evaluated exactly in that order with c0·u and c1·(…) rounded separately
 * (no contraction).  Only logical cells of `out` are written.
 */
int lhpc_stencil7_f32(const float *u, float *out, int64_t nz, int64_t ny,
                      int64_t nx, int64_t ghost, float c0, float c1,
                      int buffers_on_device, void *stream);
/* same, over z-planes [z_begin, z_end) only (halo-overlap scheduling)     */
int lhpc_stencil7_f32_planes(const float *u, float *out, int64_t nz,
                             int64_t ny, int64_t nx, int64_t ghost, float c0,
                             float c1, int64_t z_begin, int64_t z_end,
                             void *stream);
/* the three stencils with explicit variant options (NULL = automatic); the
 * stencil7 form covers planes [z_begin, z_end) of device buffers           */
int lhpc_blur_x_f32_opts(const float *a, float *b, int64_t ny, int64_t nx,
                         int64_t ghost, int nblur, int buffers_on_device,
                         void *stream, const lhpc_options *opts);
int lhpc_blur_y_f32_opts(const float *a, float *b, int64_t ny, int64_t nx,
                         int64_t ghost, int nblur, int buffers_on_device,
                         void *stream, const lhpc_options *opts);
int lhpc_stencil7_f32_planes_opts(const float *u, float *out, int64_t nz,
                                  int64_t ny, int64_t nx, int64_t ghost,
                                  float c0, float c1, int64_t z_begin,
                                  int64_t z_end, void *stream,
                                  const lhpc_options *opts);

/* ------------------------------------------- synthetic workloads (host) */
/*
 * Deterministic, thread-count-independent CSR generators (splitmix64 keyed
 * by (seed, row)), OpenMP-parallel.  See DESIGN.md §"Synthetic inputs".
 *   uniform:   every row has exactly `per_row` distinct sorted columns.
 *   powerlaw:  row lengths from a truncated discrete power law
 *              P(l) ∝ l^-alpha on [lmin, lmax]; rows 0, n/2, n-1 forced to
 *              lmax; then a seeded row shuffle.
 *   values:    U[-1,1) (dist 0) or dyadic {k/8 : k∈[-8,8]} (dist 1).
 * Two-phase: *_lengths fills row_ptr (n_rows+1, int64) and returns nnz in
 * *nnz_out; *_fill then fills col_idx (and val).
 */
int lhpc_gen_uniform_row_ptr(int64_t n_rows, int per_row, int64_t *row_ptr);
int lhpc_gen_powerlaw_row_ptr(int64_t n_rows, int64_t n_cols, double alpha,
                              int64_t lmin, int64_t lmax, uint64_t seed,
                              int64_t *row_ptr, int64_t *nnz_out);
int lhpc_gen_fill_cols(int64_t n_rows, int64_t n_cols, const int64_t *row_ptr,
                       uint64_t seed, int32_t *col_idx);
int lhpc_gen_fill_values(int dtype, int dist, int64_t count, uint64_t seed,
                         void *out);
/* int64 → int32 row_ptr narrowing (fails with LHPC_ERR_UNSUPPORTED if nnz
 * does not fit int32)                                                       */
int lhpc_row_ptr_narrow(const int64_t *in, int64_t n, int32_t *out);

/* ------------------------------------------------------------------ sort
 * LSD radix sort on the GPU, ascending, 8-bit digits over bits
 * [begin_bit, end_bit) of the key (bits outside are ignored for ordering and
 * preserved in the output).  Stable: equal keys keep their input order, so the
 * pairs variants carry values exactly like a stable CPU sort.  n < 2^32.
 * on_device = 1: keys/vals are HBM pointers and the call is asynchronous on
 * `stream` (scratch: one key + value copy, stream-ordered hipMallocAsync);
 * on_device = 0: host arrays, staged through HBM, synchronous.
 *
 * Replaces sort::gpu::radix::radix_sort(std::vector<uint32_t,…>&)
 * (reference lib/gpu/radix_gpu/src/radix_sort_gpu.cpp:24-29, the 4-pass v4
 * kernel chain lib/gpu/radix_gpu/src/cuda_radix_sort_v4.cu:17-242) — the
 * uint32 case with begin_bit = 0, end_bit = 32 — and, on the CPU side,
 * sort::radix::radix_sort (lib/sort/radix_cpu/include/radix_sort_cpu.hpp:326-331).
 */
int lhpc_radix_sort_u32(uint32_t *keys, int64_t n, int begin_bit, int end_bit,
                        int on_device, void *stream);
int lhpc_radix_sort_pairs_u32(uint32_t *keys, uint32_t *vals, int64_t n,
                              int begin_bit, int end_bit, int on_device,
                              void *stream);
int lhpc_radix_sort_pairs_u64(uint64_t *keys, uint32_t *vals, int64_t n,
                              int begin_bit, int end_bit, int on_device,
                              void *stream);

/* ------------------------------------------------------ scratch memory
 * The on-device sort, COO → CSR and CG entry points take stream-ordered
 * scratch from a library-owned pool per device (not the device's default
 * pool, so other hipMallocAsync users in the process are unaffected).  The
 * pool keeps freed scratch for the next call; lhpc_scratch_trim synchronises
 * `device` and hands the cached memory back.  lhpc_scratch_poison is test
 * support: it fills `bytes` of the current device's pool with the byte
 * `value` and frees them on `stream`, so the next scratch allocations come
 * back dirty (a kernel that reads scratch it never wrote then sees the
 * pattern).  No reference counterpart.
 */
int lhpc_scratch_trim(int device);
int lhpc_scratch_poison(int64_t bytes, int value, void *stream);

/* ------------------------------------------------------------ COO → CSR
 * Builds CSR from coordinate triples (the assembly step
 * behind sparse::to_csr(RootGrid), reference lib/sparse/include/RootGrid.hpp:20-22).
 * Entries are ordered by (row, col) with the GPU radix sort; duplicate
 * coordinates are merged by summing their values in input order (left to
 * right, in the value type).  Outputs: row_ptr (n_rows+1, int32 or int64 per
 * row_ptr_bits), col_out / val_out (capacity nnz; the first *nnz_out entries
 * are written).  Rows/cols outside [0,n_rows)/[0,n_cols) → LHPC_ERR_INVALID_ARG.
 * Synchronous (it returns the merged count).  on_device as for the sort.
 */
int lhpc_coo_to_csr(int dtype, int64_t n_rows, int64_t n_cols, int64_t nnz,
                    const int32_t *rows, const int32_t *cols, const void *vals,
                    void *row_ptr, int row_ptr_bits, int32_t *col_out,
                    void *val_out, int64_t *nnz_out, int on_device,
                    void *stream);

/* ------------------------------------------------------------------- CG
 * Conjugate gradient on an SpMV plan (no reference
 * counterpart).  lhpc_cg_solve: b and x are HBM pointers of the plan's dtype
 * (x = initial guess in, solution out); stops when ‖r‖₂ ≤ tol·‖b‖₂ (tested
 * every `check_every` iterations, the only host synchronisations) or after
 * max_iter iterations; reports the iterations run and ‖r‖/‖b‖ of the
 * recursively updated residual.  LHPC_ERR_INTERNAL on breakdown (non-finite
 * residual: the matrix is not SPD).  Dots are fp64, deterministic.  The
 * solve keeps its work (4 vectors + scalars) with the plan, and on a
 * non-null stream with check_every ≥ 4 and an ADAPTIVE plan it replays the
 * check_every iterations between two checks as a captured HIP graph, also
 * kept with the plan (results bit-identical to the loop).  So one plan
 * serves one solve at a time: a solve started while another one on the
 * same plan is running returns LHPC_ERR_BUSY (concurrent solves need a plan
 * each).  The work is allocated on the plan's device.
 * Building blocks for multi-GPU composition (all asynchronous on `stream`,
 * scalars are fp64 HBM pointers, read on the device):
 *   lhpc_vec_dot     *out = a·b
 *   lhpc_cg_step_xr  α = *alpha_num / *alpha_den; x += α·p; r -= α·q; *rr_out = r·r
 *   lhpc_cg_step_p   β = *beta_num / *beta_den; p = r + β·p
 *   lhpc_cg_step_r   α = *alpha_num / *alpha_den; r -= α·q; *rr_out = r·r
 *   lhpc_cg_step_xp  α as above, β = *beta_num / *beta_den; x += α·p; then
 *                    p = r + β·p in the same pass (beta_num NULL: x only).
 *                    step_r + step_xp = step_xr + step_p with one vector
 *                    pass less, bit-identical results.
 */
/* y = A·x and *dot_out = w·y (fp64, the stored y) in one pass for ADAPTIVE
 * plans (the CG p·q fused into the SpMV epilogue; fixed-order reduction),
 * SpMV + lhpc_vec_dot otherwise.  Device buffers, asynchronous.            */
int lhpc_spmv_dot(lhpc_spmv_plan *plan, const void *x, void *y, const void *w,
                  double *dot_out, void *stream);
int lhpc_cg_solve(lhpc_spmv_plan *plan, const void *b, void *x, double tol,
                  int max_iter, int check_every, int *iters_out,
                  double *resid_out, void *stream);
int lhpc_vec_dot(int dtype, int64_t n, const void *a, const void *b,
                 double *out, void *stream);
int lhpc_cg_step_xr(int dtype, int64_t n, const double *alpha_num,
                    const double *alpha_den, void *x, const void *p, void *r,
                    const void *q, double *rr_out, void *stream);
int lhpc_cg_step_p(int dtype, int64_t n, const double *beta_num,
                   const double *beta_den, const void *r, void *p,
                   void *stream);
int lhpc_cg_step_r(int dtype, int64_t n, const double *alpha_num,
                   const double *alpha_den, void *r, const void *q,
                   double *rr_out, void *stream);
int lhpc_cg_step_xp(int dtype, int64_t n, const double *alpha_num,
                    const double *alpha_den, const double *beta_num,
                    const double *beta_den, void *x, void *p, const void *r,
                    void *stream);

/* ------------------------------------------------------------------- I/O
 * SURVEY §8f rank 4 (the reference has no file formats).  Host-only.
 * .lcsr: 64-byte header {"LHPCCSR1", version 1, dtype, n_rows, n_cols, nnz,
 * row_ptr_bits, index_bits = 32}, then row_ptr, col_idx, val, each section
 * 64-byte aligned, little-endian.  load_header → allocate → load.
 */
int lhpc_csr_save(const char *path, int dtype, int64_t n_rows, int64_t n_cols,
                  int64_t nnz, const void *row_ptr, int row_ptr_bits,
                  const int32_t *col_idx, const void *val);
int lhpc_csr_load_header(const char *path, int *dtype, int64_t *n_rows,
                         int64_t *n_cols, int64_t *nnz, int *row_ptr_bits);
int lhpc_csr_load(const char *path, void *row_ptr, int32_t *col_idx, void *val);
/* Matrix Market "matrix coordinate {real|integer|pattern}
 * {general|symmetric|skew-symmetric}": the header gives the shape and an
 * upper bound on the expanded entry count (2× the listed entries for
 * symmetric files); read_coo fills 0-based (row, col, value-as-double)
 * triples — symmetric/skew entries expanded to both triangles, pattern
 * values 1.0 — and the count written.  Build CSR with lhpc_coo_to_csr.
 * symmetry: 0 general, 1 symmetric, 2 skew; field: 0 real, 1 integer,
 * 2 pattern.  Dense "array" and complex/hermitian files: LHPC_ERR_UNSUPPORTED. */
int lhpc_mm_read_header(const char *path, int64_t *n_rows, int64_t *n_cols,
                        int64_t *nnz_max, int *symmetry, int *field);
int lhpc_mm_read_coo(const char *path, int32_t *rows, int32_t *cols,
                     double *vals, int64_t *count);

/* --------------------------------------------------- multi-GPU (RCCL)
 * One process per GPU: each process creates one
 * communicator over RCCL (xGMI inside a node) on its device, with one
 * communication stream of its own.  Rank 0 makes the 128-byte unique id
 * (lhpc_dist_get_unique_id) and the launcher hands it to every rank (MPI,
 * torch.distributed, a file …); each rank then calls lhpc_dist_comm_create
 * with the same id.  No reference interface: the reference has no
 * multi-device code; the overlap follows its chunked
 * copy/compute pipeline (lib/gpu/transfer_overlap_testsuite/src/
 * cuda_tut_transfer_overlap.cu:41-142).
 */
#define LHPC_DIST_UNIQUE_ID_BYTES 128
typedef struct lhpc_dist_comm lhpc_dist_comm;
int lhpc_dist_get_unique_id(unsigned char *id_out /* LHPC_DIST_UNIQUE_ID_BYTES */);
int lhpc_dist_comm_create(lhpc_dist_comm **out, const unsigned char *id, int nranks, int rank,
                          int device);
int lhpc_dist_comm_info(const lhpc_dist_comm *comm, int *nranks, int *rank, int *device);
int lhpc_dist_comm_destroy(lhpc_dist_comm *comm);
/* in-place sum over ranks of `count` doubles (the CG dots), async on
 * stream: ncclAllReduce, or over a P2P communicator (lhpc_dist_comm_create_local,
 * after a window import) every rank's values gathered through the flag
 * allocation's scalar slots and added in rank order (count ≤ 8).
 * lhpc_dist_allgather_f64: out[r·count + i] = rank r's vals[i] (same paths)  */
int lhpc_dist_allreduce_sum_f64(lhpc_dist_comm *comm, double *buf, int64_t count, void *stream);
int lhpc_dist_allgather_f64(lhpc_dist_comm *comm, const double *vals, int64_t count, double *out, void *stream);
/*
 * Distributed y = A·x.  The n_rows rows are cut into nranks·K blocks by
 * `cuts` (nranks·K + 1 ascending global rows, cuts[0] = 0; nnz-balanced:
 * lhpc_csr_partition_rows(row_ptr, bits, n_rows, nranks·K, cuts)); block
 * b = k·nranks + r belongs to rank r as its chunk k.  Each rank passes its
 * LOCAL CSR: its K blocks stacked in chunk order (row_ptr rebased to 0,
 * global column indices, host arrays, copied to HBM).  lhpc_dist_spmv reads
 * the full x (n_cols, device) and leaves the full y (n_rows, device, not x)
 * on every rank: chunk k is reduced into this rank's rows of y, then the
 * comm stream delivers every rank's block of chunk k while the compute
 * stream reduces chunk k+1: one in-place ncclAllGather when chunk k's
 * blocks are all the same size (uniform rows), else a group of in-place
 * ncclBroadcast (one per root, exact slices).
 * Asynchronous on `stream`.  Matrices that do not select the XTILE layout
 * use one plan per block.
 */
typedef struct lhpc_dist_spmv_plan lhpc_dist_spmv_plan;
int lhpc_dist_spmv_plan_create(lhpc_dist_spmv_plan **out, lhpc_dist_comm *comm, int dtype, int64_t n_rows,
                          int64_t n_cols, int K, const int64_t *cuts, const void *row_ptr,
                          int row_ptr_bits, const int32_t *col_idx, const void *val, unsigned flags);
/* the same with explicit options (NULL = automatic): the local plans' SpMV
 * variant fields and the dist_* fields (exchange kind, broadcast groups)   */
int lhpc_dist_spmv_plan_create_opts(lhpc_dist_spmv_plan **out, lhpc_dist_comm *comm, int dtype,
                                    int64_t n_rows, int64_t n_cols, int K, const int64_t *cuts,
                                    const void *row_ptr, int row_ptr_bits, const int32_t *col_idx,
                                    const void *val, unsigned flags, const lhpc_options *opts);
int lhpc_dist_spmv(lhpc_dist_spmv_plan *d, const void *x, void *y, void *stream);
/*
 * Cross-step overlap for iterative use (y of call n is x of call n+1).
 * lhpc_dist_spmv = lhpc_dist_spmv_begin + lhpc_dist_spmv_end.  _begin issues
 * the call but leaves the exchange of y in flight (y is NOT complete on
 * `stream` afterwards); _end makes `stream` wait for it.  When the x of a
 * _begin is the y of the previous _begin on this plan, the x tiles are
 * gathered by column part: chunk j's rows of y are one contiguous column
 * range of the next x (square matrices), so the gather of the tiles inside
 * it waits only for exchange j of the previous call and runs while the
 * later chunks still travel (lhpc_dist_chain_parts gives the tile → chunk
 * map).  Any other x first finishes the pending call.  P2P windows signal
 * DONE per chunk for this (flag value epoch·64 + chunk + 1; K ≤ 63).
 * Anchor: the chunked copy/compute overlap of the reference's
 * lib/gpu/transfer_overlap_testsuite/src/cuda_tut_transfer_overlap.cu:41-142,
 * carried across steps.
 */
int lhpc_dist_spmv_begin(lhpc_dist_spmv_plan *d, const void *x, void *y, void *stream);
int lhpc_dist_spmv_end(lhpc_dist_spmv_plan *d, void *stream);
/* the rank's local plan (the row-range plan over its K blocks, else its
 * first block's plan) and whether chained calls gather by column part      */
int lhpc_dist_spmv_plan_info(const lhpc_dist_spmv_plan *d, lhpc_spmv_plan_info *info, int *chained_stage);
/* host only: part[t] for each of the n_tiles x tiles of tile_width columns =
 * the first exchange chunk j whose end row cuts[(j+1)·nranks] covers the
 * tile's last column (the order chunks land in) */
int lhpc_dist_chain_parts(const int64_t *cuts, int nranks, int K, int64_t n_cols, int64_t tile_width,
                          int32_t *part, int64_t n_tiles);
/* the exchange of a whole call alone (every chunk, no SpMV): y must already
 * hold this rank's blocks; for exchange-only timing (bench.py --gpus N)    */
int lhpc_dist_exchange(lhpc_dist_spmv_plan *d, void *y, void *stream);
/*
 * Conjugate gradient over a distributed plan (SURVEY §8f rank 3 with the
 * multi-GPU path; square SPD matrix).  b, x and p_work are full-length
 * (n_rows) device vectors of the plan's dtype on this rank's device: b is
 * read on this rank's rows, x is the initial guess (complete on every rank)
 * and on return holds the whole solution on every rank, p_work is the search
 * direction — register it as a P2P window (lhpc_dist_p2p_export/_import) to
 * exchange it by peer stores, else the plan's RCCL exchange.  Per iteration:
 * q = A·p on this rank's rows (a chained stage: part j of p is gathered as
 * soon as exchange j of p has landed), the dots p·q and r·r as K block
 * partials per rank all-gathered and added in global block order (so the
 * solve is independent of how the same block split is spread over ranks),
 * the fused x/r/p updates on this rank's rows, and the exchange of p's
 * blocks.  K ≤ 8.  Stops as lhpc_cg_solve; LHPC_ERR_INTERNAL on breakdown or
 * a timed-out P2P flag wait.  Synchronous (host checks every check_every).
 */
int lhpc_dist_cg_solve(lhpc_dist_spmv_plan *d, const void *b, void *x, void *p_work, double tol,
                       int max_iter, int check_every, int *iters_out, double *resid_out, void *stream);
int lhpc_dist_spmv_plan_destroy(lhpc_dist_spmv_plan *d);
/*
 * The exchange schedule of lhpc_dist_spmv, as data (host only; the call
 * issues exactly these transfers, in this order, per chunk k):
 *   LHPC_XFER_ALLGATHER  chunk k's nranks blocks are equal (count rows each):
 *                        one in-place all-gather of y[offset, offset +
 *                        nranks·count), this rank sending y[send_offset, +count)
 *   LHPC_XFER_BROADCAST  unequal blocks (or dist_broadcast): one in-place
 *                        broadcast from `root` of y[offset, offset + count) per
 *                        non-empty block, inside one group per chunk
 *   LHPC_XFER_PUSH       peer exchange: this rank stores y[offset, +count)
 *                        (its own block) into every peer's y
 * Offsets and counts are in elements of y.  exchange: LHPC_DIST_EXCHANGE_RCCL
 * or _P2P; broadcast: 1 = broadcast groups even for equal blocks.
 * Returns the number of entries in *n_out (capacity max_out; LHPC_ERR_INVALID_ARG
 * if too small).  Replaces nothing in the reference (no collectives there).
 */
enum lhpc_xfer_kind { LHPC_XFER_ALLGATHER = 1, LHPC_XFER_BROADCAST = 2, LHPC_XFER_PUSH = 3 };
typedef struct lhpc_dist_xfer {
  int32_t chunk;
  int32_t kind;                 /* enum lhpc_xfer_kind                           */
  int32_t root;                 /* broadcast root / pushing rank (−1: all-gather) */
  int32_t group;                /* 1 when the entry is inside a chunk's group    */
  int64_t offset;               /* first element of y the transfer fills          */
  int64_t count;                /* elements (all-gather: per rank)               */
  int64_t send_offset;          /* all-gather: this rank's contribution           */
} lhpc_dist_xfer;
int lhpc_dist_exchange_schedule(const int64_t *cuts, int nranks, int K, int rank, int exchange,
                                int broadcast, lhpc_dist_xfer *out, int64_t max_out, int64_t *n_out);
/*
 * The RCCL calls themselves, argument by argument, that the RCCL exchange
 * issues for this rank (lhpc_dist_spmv, one process per rank) or device
 * (the single-process multi-device plan, device index = rank): both device
 * paths walk exactly this list (lhpc_rccl.hpp), the CPU tests check it for
 * every rank against RCCL's contracts (matching collectives on every rank,
 * the in-place all-gather's sendbuff == recvbuff + rank·count, broadcast
 * roots) and emulate it.  One entry per call, chunk order:
 *   op  LHPC_RCCL_ALLGATHER: ncclAllGather(y + send_byte_offset,
 *       y + recv_byte_offset, count, datatype, comm, stream);
 *       LHPC_RCCL_BROADCAST: ncclBroadcast(y + send_byte_offset,
 *       y + recv_byte_offset, count, datatype, root, comm, stream)
 *   group_begin / group_end: ncclGroupStart() before / ncclGroupEnd() after
 *       the call (lhpc_dist_spmv; the multi-device plan brackets each chunk's
 *       calls of all its devices in one group instead)
 * datatype is the ncclDataType_t value (ncclFloat32 / ncclFloat64).
 */
enum lhpc_rccl_op { LHPC_RCCL_ALLGATHER = 1, LHPC_RCCL_BROADCAST = 2 };
typedef struct lhpc_rccl_call {
  int32_t chunk;
  int32_t op;                   /* enum lhpc_rccl_op                              */
  int32_t root;                 /* broadcast root (−1: all-gather)                */
  int32_t datatype;             /* ncclDataType_t                                 */
  int32_t group_begin;          /* ncclGroupStart() before this call              */
  int32_t group_end;            /* ncclGroupEnd() after this call                 */
  int64_t send_byte_offset;     /* sendbuff = (char *)y + send_byte_offset         */
  int64_t recv_byte_offset;     /* recvbuff = (char *)y + recv_byte_offset         */
  int64_t count;                /* elements (all-gather: per rank)                */
} lhpc_rccl_call;
int lhpc_dist_rccl_calls(const int64_t *cuts, int nranks, int K, int rank, int broadcast, int dtype,
                         lhpc_rccl_call *out, int64_t max_out, int64_t *n_out);
/*
 * Direct peer exchange of y (SURVEY §8e "Optimisation": every pair of
 * MI355X in a node is connected by xGMI).  Each rank exports a y buffer
 * (device, ≥ n_rows values, 4-byte multiple) as a blob of IPC handles, the
 * launcher all-gathers the blobs (any channel, rank order) and every rank
 * imports them.  Up to LHPC_DIST_P2P_MAX_WINDOWS windows per communicator
 * (export/import them in the same order on every rank): with two, the
 * iterative loop's ping-pong pair (y of call n is x of call n+1) gets peer
 * stores on every call.  lhpc_dist_spmv with y equal to a window then pushes
 * each chunk's block into every peer's copy of that window with one kernel
 * (stores over xGMI, all links at once) instead of RCCL collectives; per
 * call a READY flag ("my y may be overwritten": issued on the call's
 * stream, so prior work on it that reads y is done) and a DONE flag ("my
 * pushes have landed") go to every peer, and the comm stream waits for all
 * peers' flags with a bounded spin.  A spin that times out sets the
 * communicator's status word: the pushes and DONE of that call are then
 * skipped on the device and every later call fails — check
 * lhpc_dist_p2p_status after synchronising the stream.  y must not be read
 * by any stream other than the call's until the call completes.  Without
 * RCCL, lhpc_dist_comm_create_local gives a communicator for this exchange
 * only (lhpc_dist_allreduce_sum_f64 / stencil7 need RCCL:
 * LHPC_ERR_UNSUPPORTED).  The exchange kind is a plan option
 * (lhpc_options.dist_exchange; automatic = peer stores for a window).
 */
#define LHPC_DIST_P2P_BLOB_BYTES 192
#define LHPC_DIST_P2P_MAX_WINDOWS 4
int lhpc_dist_comm_create_local(lhpc_dist_comm **out, int nranks, int rank, int device);
int lhpc_dist_p2p_export(lhpc_dist_comm *comm, void *y, int64_t bytes,
                         unsigned char *blob_out /* LHPC_DIST_P2P_BLOB_BYTES */);
int lhpc_dist_p2p_import(lhpc_dist_comm *comm,
                         const unsigned char *blobs /* nranks × LHPC_DIST_P2P_BLOB_BYTES */);
/* lhpc_dist_p2p_unmap: undoes the LAST window (y must be its buffer) on this
 * rank — peer mappings closed, the window dropped whether it was imported or
 * only exported — after synchronising the comm stream.  A setup whose import
 * failed on any rank calls it on every rank that exported, so window indices
 * stay aligned across ranks and no rank keeps a window its peers never mapped.
 * lhpc_dist_p2p_reset unmaps every window and frees this rank's flag array.
 * It is COLLECTIVE: every rank resets (peers still hold this rank's flag
 * array mapped), with a barrier before any rank exports again.  Blobs carry a
 * flags generation, so an import after a reset remaps the peers' new flag
 * arrays instead of trusting the old mapping.                              */
int lhpc_dist_p2p_unmap(lhpc_dist_comm *comm, void *y);
int lhpc_dist_p2p_reset(lhpc_dist_comm *comm);
int lhpc_dist_p2p_status(const lhpc_dist_comm *comm);
/*
 * One 7-point stencil step on this rank's z-slab (BASELINE config C5): u and
 * out are HPCHighDimensionFlatArray<3,float,ghost> buffers of logical
 * (nzl, ny, nx) on the device; the z ghost planes -1 and nzl of u are the
 * halo, refreshed from the neighbouring ranks (ncclSend/ncclRecv of the
 * boundary planes on the comm stream) while the interior planes run; the
 * first and last rank keep their outer ghost planes (Dirichlet).  Bit-exact
 * with the single-domain lhpc_stencil7_f32.  Asynchronous on `stream`.
 */
int lhpc_dist_stencil7_f32(lhpc_dist_comm *comm, float *u, float *out, int64_t nzl, int64_t ny,
                           int64_t nx, int64_t ghost, float c0, float c1, void *stream);
/* The same step with the halo exchange chosen (enum lhpc_dist_exchange):
 * RCCL (send/recv, as above) or P2P — u is a registered window on every rank
 * (lhpc_dist_p2p_export/_import, windows may differ in size: slabs of
 * different depth) and each rank stores its boundary planes straight into
 * its neighbours' ghost planes over xGMI, under the READY/DONE flags of the
 * SpMV windows (neighbours only); the boundary planes wait for the
 * neighbours' DONE on `stream`.  AUTO: P2P when u is a window, else RCCL.
 * In a time loop register both ping-pong buffers.                          */
int lhpc_dist_stencil7_f32_x(lhpc_dist_comm *comm, float *u, float *out, int64_t nzl, int64_t ny,
                             int64_t nx, int64_t ghost, float c0, float c1, int exchange, void *stream);

#ifdef __cplusplus
} /* extern "C" */
#endif
#endif /* LHPC_H_ */
