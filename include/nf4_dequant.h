/*
 * nf4_dequant.h -- C ABI of the MI355X (gfx950) NF4 double-dequantization path.
 *
 * Library: nf4_triton_dequantization_amd/_lib/libnf4dq.so (hipcc, gfx950).
 * Every entry point is asynchronous on the given HIP stream, allocates nothing,
 * keeps no global mutable state, and returns 0 or an NF4DQ_* error code.
 * Pointers are device pointers unless stated otherwise; `hip_stream` is a
 * hipStream_t (NULL = the null stream).
 *
 * Reference interfaces replaced (felipemcoelho/nf4-triton-dequantization,
 * file nf4_triton_dequantization/kernel_optimized.py):
 *   nf4_dequant_ref    <- _triton_dequantize_main :142-205 launching
 *                         _nf4_dequantize_kernel_final :11-110 (uint8 absmax,
 *                         double dequant; wrap/truncate rules :173-186)
 *   nf4_dequant_single <- the non-uint8 absmax branch :166-167 -> :273-274
 *   nf4_dequant_ref_batched <- benchmark.py:68-84 (several Linear4bit weights
 *                         per step) folded into one launch
 *   nf4_dequant_ref_cpu / nf4_dequant_single_cpu <- _aggressive_pytorch_t4
 *                         :208-314, the reference's CPU path (HOST pointers,
 *                         synchronous, `threads` worker threads)
 *   nf4_dequant_bnb / nf4_dequant_bnb_single <- bitsandbytes dequantize_4bit
 *                         semantics; the reference
 *                         never implements these, they are parity-unpinned.
 */
#ifndef NF4_DEQUANT_H_
#define NF4_DEQUANT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Output dtypes (quant_state.dtype, kernel_optimized.py:123, :189). */
#define NF4DQ_F16 0
#define NF4DQ_BF16 1
#define NF4DQ_F32 2

/* Return codes. HIP launch failures are NF4DQ_ERR_HIP_BASE + hipError_t. */
#define NF4DQ_OK 0
#define NF4DQ_ERR_ARG 1        /* null pointer, bad dtype, negative size      */
#define NF4DQ_ERR_SHAPE 2      /* sizes the reference would reject (view fails) */
#define NF4DQ_ERR_TOO_LARGE 3  /* a single matrix beyond 2^31 packed bytes    */
#define NF4DQ_ERR_SPLITK_TIMEOUT 4 /* nf4_gemm_check_workspace: a split-K reducer gave up */
#define NF4DQ_ERR_HIP_BASE 1000

/* Reference double dequant of one Linear4bit weight into row-major out[m][n].
 *   packed   uint8[packed_len]  two NF4 codes per byte, high nibble first;
 *                               row r starts at r*(packed_len/m)
 *   absmax_q uint8[nb]          per (row, 64-column block); index wraps mod nb
 *   absmax2  fp32[n2]           index r*ceil(bpr/4) + block/4, wraps mod n2
 * out[r][c] = RNE(NF4[nib] * ((float)absmax_q[.] / 127.0f * absmax2[.])).
 * Errors: packed_len % m != 0 or packed_len/m < ceil(n/2) -> NF4DQ_ERR_SHAPE.
 *
 * Departure from SURVEY.md §8(b): the survey's contract is
 *   nf4_dequant_ref(packed, absmax_q, nb, absmax2, n2, out, out_dtype, m, n, hip_stream);
 * this entry (and nf4_dequant_ref_cpu, nf4_dequant_single, nf4_dequant_single_cpu)
 * adds `packed_len` right after `packed`.  The reference reads the packed weight as
 * `weight.data.view(m, -1)` (kernel_optimized.py:229), so the row stride is
 * numel / m -- padded rows and odd widths included (:288-312) -- and a pointer
 * alone does not carry numel.  Without it the ABI could only assume the dense
 * stride ceil(n/2) and would silently misread padded weights the reference
 * accepts; with it, sizes the reference's view would reject are NF4DQ_ERR_SHAPE. */
int nf4_dequant_ref(const uint8_t* packed, int64_t packed_len,
                    const uint8_t* absmax_q, int64_t nb,
                    const float* absmax2, int64_t n2,
                    void* out, int32_t out_dtype, int64_t m, int64_t n,
                    void* hip_stream);

/* Single-quant branch: absmax fp32[absmax_len] viewed as [m, absmax_len/m],
 * scale of (r, b) = absmax[r*(absmax_len/m) + b]. */
int nf4_dequant_single(const uint8_t* packed, int64_t packed_len,
                       const float* absmax, int64_t absmax_len,
                       void* out, int32_t out_dtype, int64_t m, int64_t n,
                       void* hip_stream);

/* Host-CPU forms of nf4_dequant_ref / nf4_dequant_single:
 * same arguments, same semantics bit for bit, same error codes, but every
 * pointer is a HOST pointer and the call is synchronous; `threads` worker
 * threads split the rows (<= 0 = all hardware threads).  AVX2 table lookups
 * when the CPU has AVX2, a scalar loop otherwise (same results).  Replaces the
 * reference's CPU fallback _aggressive_pytorch_t4 (kernel_optimized.py:208-314). */
int nf4_dequant_ref_cpu(const uint8_t* packed, int64_t packed_len,
                        const uint8_t* absmax_q, int64_t nb,
                        const float* absmax2, int64_t n2,
                        void* out, int32_t out_dtype, int64_t m, int64_t n,
                        int32_t threads);
int nf4_dequant_single_cpu(const uint8_t* packed, int64_t packed_len,
                           const float* absmax, int64_t absmax_len,
                           void* out, int32_t out_dtype, int64_t m, int64_t n,
                           int32_t threads);

/* One matrix of a batched call (host memory; copied into kernel arguments). */
typedef struct nf4_matrix_desc {
    const uint8_t* packed;
    int64_t packed_len;
    const uint8_t* absmax_q;
    int64_t nb;
    const float* absmax2;
    int64_t n2;
    void* out;
    int64_t m;
    int64_t n;
} nf4_matrix_desc;

/* Dequantize `count` matrices (same out_dtype) with as few launches as the
 * kernel-argument budget allows (NF4DQ_BATCH_MAX matrices per launch). */
#define NF4DQ_BATCH_MAX 24
int nf4_dequant_ref_batched(const nf4_matrix_desc* descs, int32_t count,
                            int32_t out_dtype, void* hip_stream);

/* bitsandbytes nested semantics over the flat element stream:
 *   absmax_f32[i] = code2[absmax_q[i]] * absmax2[i / blocksize2] + offset
 *   out[k]        = RNE(NF4[nib(k)] * absmax_f32[k / blocksize])
 * blocksize and blocksize2 must be powers of two, blocksize >= 64. */
int nf4_dequant_bnb(const uint8_t* packed, const uint8_t* absmax_q, int64_t nb,
                    const float* code2, const float* absmax2, int64_t n2,
                    float offset, void* out, int32_t out_dtype, int64_t numel,
                    int32_t blocksize, int32_t blocksize2, void* hip_stream);

/* bitsandbytes single-level (compress_statistics=False): fp32 absmax per block. */
int nf4_dequant_bnb_single(const uint8_t* packed, const float* absmax, int64_t nabs,
                           void* out, int32_t out_dtype, int64_t numel,
                           int32_t blocksize, void* hip_stream);

/* Launch tuning (bench/tuning only; the entry points above use the default
 * {4, 0, 1, 0}).  tile_dwords must be 4 and nontemporal 1 (the tile shape and
 * the sc1+nt output stores every entry point uses; the other shapes and store
 * policies measured slower and were removed, profiles/r01/tune_sweep.log,
 * profiles/r02/x4_direct/).  blocks_per_cu: grid cap per CU (0 = one wave per
 * tile, no cap; capped grids walk tiles persistently).  flags: 0, or one of
 * NF4DQ_CFG_CHUNKS (the matrix goes through the path of every shape the flat
 * kernel does not take -- n % 64 != 0, padded rows, unaligned pointers: the chunk
 * kernels and, since round 6, the piece kernels -- even when it is flat-eligible) or
 * NF4DQ_CFG_ROWS (through the one-thread-per-byte general kernel, which otherwise
 * runs only past the chunk kernel's 32-bit index limits); for tests and tuning.
 * Other bits: NF4DQ_ERR_ARG.
 * (Absmax-line and page-translation prefetches were tried as flags and measured
 * no better than 1 %, profiles/r03/c5/; removed.) */
#define NF4DQ_CFG_ROWS 1
#define NF4DQ_CFG_CHUNKS 2
typedef struct nf4_launch_cfg {
    int32_t tile_dwords;
    int32_t blocks_per_cu;
    int32_t nontemporal;
    int32_t flags;
} nf4_launch_cfg;

int nf4_dequant_ref_cfg(const uint8_t* packed, int64_t packed_len,
                        const uint8_t* absmax_q, int64_t nb,
                        const float* absmax2, int64_t n2,
                        void* out, int32_t out_dtype, int64_t m, int64_t n,
                        const nf4_launch_cfg* cfg, void* hip_stream);

/* Fused dequant + GEMM for small M (decode-shaped activations; replaces the
 * reference harness's `X @ triton_dequantize_nf4(W).t()`, benchmark.py:61-66):
 *   y[M][N] = x[M][K] . W[N][K]^T,  W = the weights nf4_dequant_ref would
 *   write (reference semantics, bit-identical), fp32 accumulation (MFMA).
 * x, y: fp16/bf16 (out_dtype), row-major.  Fast-path shape rules (else
 * NF4DQ_ERR_SHAPE): M <= NF4DQ_GEMM_MAX_M, N % 64 == 0, K % 128 == 0,
 * packed_len == N*K/2 (and N <= 2^18).  `workspace` (16-byte aligned) must hold
 * nf4_gemm_workspace_bytes(M, N, K) bytes (0 = none needed): split-K ticket
 * counters + 64-bit partial-sum entries, handed between workgroups with relaxed
 * agent-scope atomics only and reduced inside the launch in a fixed order
 * (bitwise reproducible).  The workspace must be ZERO-FILLED before its first
 * use; every call leaves it reusable (counters and entries back to 0).  One
 * workspace per stream: concurrent calls must not share one. */
#define NF4DQ_GEMM_MAX_M 32
size_t nf4_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K);
int nf4_gemm_ref(const void* x, int64_t M, const uint8_t* packed, int64_t packed_len,
                 const uint8_t* absmax_q, int64_t nb, const float* absmax2, int64_t n2,
                 void* y, int32_t out_dtype, int64_t N, int64_t K,
                 void* workspace, size_t workspace_bytes, void* hip_stream);

/* Tuning form of nf4_gemm_ref.  kernel: 0 = library choice,
 * NF4DQ_GEMM_STREAM (K % 256 == 0; waves 4/8/16, depth = chunks in flight per
 * wave 2/4/8 (8 not with 16 waves; 16 waves only when M <= 16), strips = 16-column strips per workgroup
 * 1/2/4 dividing waves) or NF4DQ_GEMM_K128 (waves 4/8, depth 1/2/4 (<= 2 when
 * M > 16), strips = 16-column strips per wave 1/2/4 (0 = 1), sharing x loads).  ksplit: K slices reduced across workgroups.
 * NF4DQ_GEMM_PERSIST: the streaming kernel's persistent form (M <= 16,
 * ksplit 1..16 K slices dividing K / 256, waves / strips K parts dividing a slice into a multiple of depth
 * (2/4), x[M][K] in LDS, absmax not wrapping inside a row).
 * An invalid combination returns NF4DQ_ERR_ARG. */
#define NF4DQ_GEMM_K128 1
#define NF4DQ_GEMM_STREAM 2
#define NF4DQ_GEMM_PERSIST 3
/* NF4DQ_GEMM_XS: shared-activation kernel (any M <= 32, K % 128 == 0): a
 * workgroup of `waves` (4/8) waves owns one 16-column strip per wave over a K
 * slice of `depth` (2/4/8) 128-deep chunks, the x slice staged once in LDS and
 * every weight chunk in flight at once; ksplit must equal ceil(K/128 / depth);
 * strips 0 or 1. */
#define NF4DQ_GEMM_XS 4
/* NF4DQ_GEMM_XR: register-resident activation kernel (any M <= 32, K % 128 ==
 * 0): the K split is over the `waves` (8/16) waves of a workgroup, each holding
 * its x fragments of `strips` 128-deep chunks in registers for the whole
 * launch; a workgroup walks its column strips with a `depth` (2/4) deep ring of
 * weight loads and sums the waves' partial tiles in LDS; `strips` = 128-deep
 * chunks per wave: 1, 2 (one 256-deep chunk, K % 256 == 0) or 4 (two, 8 waves
 * only, K % 512 == 0); ksplit must equal ceil(K/128 / (waves * strips))
 * (1 = no cross-workgroup reduction). */
#define NF4DQ_GEMM_XR 5
/* NF4DQ_GEMM_SK (6): retired in round 6.  The balanced ("stream-K") kernel was
 * never the library's choice (slower than the persistent kernel at every measured
 * shape) and no longer ships; a cfg naming it is rejected with NF4DQ_ERR_ARG. */
#define NF4DQ_GEMM_SK 6
/* NF4DQ_GEMM_GEMV: the decode GEMV (M == 1, K % 2048 == 0, K <= 16384, absmax not
 * wrapping inside a row): no MFMA; a lane dots 32 consecutive exact weights of a row
 * with x on the VALU.  waves 8/16 per workgroup, depth = rows per row group 1/2/4,
 * ksplit 1, strips = workgroups per CU 0/1/2 (0 = 1).  The library's choice at M = 1
 * for launches of up to 4096 columns. */
#define NF4DQ_GEMM_GEMV 7
typedef struct nf4_gemm_cfg {
    int32_t kernel;
    int32_t waves;
    int32_t depth;
    int32_t ksplit;
    int32_t strips;
} nf4_gemm_cfg;
size_t nf4_gemm_workspace_bytes_cfg(int64_t M, int64_t N, int64_t K, const nf4_gemm_cfg* cfg);
int nf4_gemm_ref_cfg(const void* x, int64_t M, const uint8_t* packed, int64_t packed_len,
                     const uint8_t* absmax_q, int64_t nb, const float* absmax2, int64_t n2,
                     void* y, int32_t out_dtype, int64_t N, int64_t K,
                     void* workspace, size_t workspace_bytes, const nf4_gemm_cfg* cfg, void* hip_stream);

/* Several weights that share the activation x (q/k/v, gate/up): one launch.
 * Each weight: packed [N*K/2], its own absmax_q / absmax2 (reference wrap
 * semantics per weight), output y [M][N] (out_dtype).  Same shape rules as
 * nf4_gemm_ref for every weight (N % 64 == 0), at most NF4DQ_GEMM_GROUP_MAX
 * weights; cfg NULL = library choice for the summed N.  Every kernel runs
 * the group as one launch (the library's persistent choice falls back to one
 * launch per weight when absmax wraps inside a row).  Workspace as for
 * nf4_gemm_ref, sized by nf4_gemm_grouped_workspace_bytes. */
#define NF4DQ_GEMM_GROUP_MAX 8
typedef struct nf4_gemm_mat {
    const uint8_t* packed;
    int64_t packed_len;
    const uint8_t* absmax_q;
    int64_t nb;
    const float* absmax2;
    int64_t n2;
    void* y;
    int64_t N;
} nf4_gemm_mat;
size_t nf4_gemm_grouped_workspace_bytes(int64_t M, int64_t K, const nf4_gemm_mat* mats, int32_t count,
                                        const nf4_gemm_cfg* cfg);
int nf4_gemm_ref_grouped(const void* x, int64_t M, int64_t K, const nf4_gemm_mat* mats, int32_t count,
                         int32_t out_dtype, void* workspace, size_t workspace_bytes,
                         const nf4_gemm_cfg* cfg, void* hip_stream);

/* The split-K hand-off never hangs: a reducer that has polled a partner slice's
 * entries 2^16 times without seeing them gives up, reads them as NaN and sets a
 * sticky error word in the workspace header.  This call waits for `hip_stream`,
 * reads that word and returns NF4DQ_OK, or NF4DQ_ERR_SPLITK_TIMEOUT after
 * zero-filling the whole workspace again (a stalled slice's late entries
 * included), so it is reusable.  NULL / 0-byte workspace: NF4DQ_OK (no split-K,
 * nothing to report).  Synchronous; call it after the calls it vouches for. */
int nf4_gemm_check_workspace(void* workspace, size_t workspace_bytes, void* hip_stream);

/* Human-readable text for a return code (static storage). */
const char* nf4_strerror(int code);

/* Library version string, e.g. "nf4dq 0.1.0 gfx950". */
const char* nf4_version(void);

#ifdef __cplusplus
}
#endif

#endif /* NF4_DEQUANT_H_ */
