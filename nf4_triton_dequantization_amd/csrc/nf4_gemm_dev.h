// nf4_gemm_dev.h -- fused NF4 dequant + GEMM for small M (decode-shaped
// activations): Y[M, N] = X[M, K] . W[N, K]^T with W in the bitsandbytes NF4
// layout, reference double-dequant semantics (the same bf16/fp16 weights
// nf4_dequant_ref would materialise, bit for bit), fp32 accumulation on MFMA.
//
// What it replaces: the consumer pattern of the reference harness,
// `X @ triton_dequantize_nf4(W).t()` (benchmark.py:61-66), which writes the
// dequantized weight to HBM and reads it back.  Here the 4-bit weight is read
// once (0.5 B/element) and dequantized in registers -- the roofline is HBM on
// the packed weight, not on a 2 B/element bf16 copy.
//
// Six kernels (host choice in default_gemm_cfg, explicit in nf4_gemm_ref_cfg):
//  * nf4_gemm_smallm_kernel -- K % 128 == 0; 128-deep chunks, a lane loads 16
//    packed bytes of its weight row (one 64-block, one scale) and the matching
//    activation fragments from global memory; waves of a workgroup split K and
//    meet in LDS.  The fallback for any shape the others do not take.
//  * nf4_gemm_xs_kernel -- shared-activation form of the 128-deep kernel: the
//    x slice staged once per workgroup in LDS, one strip per wave.
//  * nf4_gemm_xr_kernel -- register-resident x (16 < M <= 32, K % 256 == 0):
//    each wave holds its K chunk's x fragments for the whole launch and walks
//    the workgroup's column strips with a register ring of weight chunks.
//  * nf4_gemm_xrg_kernel -- the same body with the reduction groups unrolled
//    (two K slices, <= 16 strips per workgroup): each group's split-K exchanges
//    go out inside the strip loop (up to 2 waves per SIMD, 256 registers).
//  * nf4_gemm_stream_kernel -- K % 256 == 0 (every Llama shape); 256-deep
//    chunks (one 128-byte line per weight row), activations staged in LDS,
//    a register ring of weight chunks, pair-table dequant (see its comments).
//  * nf4_gemm_persist_kernel -- the streaming body with one workgroup per CU
//    walking strip groups (M <= 16), the ring running on across groups.
// (The seventh, the decode GEMV for M = 1 -- no MFMA, the exact weights dotted with x on
// the VALU -- lives with its launcher in nf4_gemm_launch_gemv.hip.)
// All use the same k permutation on A and B fragments (a lane's packed dword
// is exactly its MFMA B fragment of one step), so no shuffle is needed.  K
// slices over workgroups (ksplit > 1) write fp32 partials to a workspace slab;
// the last workgroup to finish a column strip (ticket counter) sums the slices
// in slice order and writes y -- one launch, bitwise reproducible, no float atomics.
// Device side of the fused GEMM: helpers, the split-K hand-off and the kernel
// templates.  Shared by the host dispatch (nf4_gemm.hip) and one launcher source
// per kernel family (nf4_gemm_launch_*.hip), which instantiate the kernels they
// launch -- the families compile in parallel.  Everything here has internal
// linkage (anonymous namespace), so every source gets its own copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nf4_dequant.h"
#include "nf4_common.h"

namespace {

using namespace nf4dq;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kOob = 0x80000000u;  // beyond every buffer range: loads return 0, stores drop

// Phase-stamp hooks: empty in the library.  tools/gemm_stamps.hip defines them
// (per-wave s_memrealtime stamps into a buffer of its own) and includes this file
// to build the diagnostic library tools/_build/libnf4dq_gstamps.so; nothing in
// the product reads or writes a stamp.
//   NF4_GSTAMP(slot)          the wave's time at this point
//   NF4_GSPAN_BEGIN()         start of a repeated span (e.g. one reduction barrier)
//   NF4_GSPAN_END(slot)       add the span's length to slot
#ifndef NF4_GSTAMP
#define NF4_GSTAMP(slot_) ((void)0)
#define NF4_GSPAN_BEGIN() ((void)0)
#define NF4_GSPAN_END(slot_) ((void)0)
#define NF4_GSTAMP_INIT(waves_) ((void)0)
#endif

// Ablation hooks of the pair-table kernels (register-resident, streaming,
// persistent): the product operation by default.  tools/gemm_ablate.hip redefines
// them to time a kernel with one part removed (its results are then wrong: timing
// only, never in the library).
//   NF4_ABL_LOOKUP(pt, addr, wd)  pair-table read of the two codes of a byte
//   NF4_ABL_WLOAD(rsrc, off)      16-byte weight load of the ring
//   NF4_ABL_MMA_ON                the MFMAs (operands kept alive when off)
//   NF4_ABL_RED_ON / _HANDOFF_ON  register-resident kernel: in-LDS K reduction / split-K hand-off
//   NF4_ABL_X_ON                  register-resident kernel: the x fragments' global loads
//   NF4_ABL_SLOAD(rsrc, off, b8)  register-resident kernel: absmax byte / nested scale gather
#ifndef NF4_ABL_X_ON
#define NF4_ABL_X_ON 1
#endif
#ifndef NF4_ABL_XFRAG  // the streaming / persistent body's x fragment (an LDS read)
#define NF4_ABL_XFRAG(smem_, off_) (*reinterpret_cast<const u32x4*>((smem_) + (off_)))
#endif
#ifndef NF4_ABL_SLOAD
#define NF4_ABL_SLOAD(rsrc_, off_, b8_)                                                       \
    ((b8_) ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8((rsrc_), (off_), 0, 0) \
           : __builtin_amdgcn_raw_buffer_load_b32((rsrc_), (off_), 0, 0))
#endif
#ifndef NF4_ABL_LOOKUP
#define NF4_ABL_LOOKUP(pt_, addr_, wd_) (*reinterpret_cast<const f32x2*>((pt_) + (addr_)))
#endif
#ifndef NF4_ABL_WLOAD
#define NF4_ABL_WLOAD(rsrc_, off_) __builtin_amdgcn_raw_buffer_load_b128((rsrc_), (off_), 0, 0)
#endif
//   NF4_ABL_KEEP_SLICE(ks)        128-deep kernel: K slice ks stores its split-K partials
//                                 (tools' drop-slice build withholds one slice's: the
//                                 reducer's poll then gives up and sets the error word)
//   NF4_ABL_RING_FULL             0 when the ring issues fewer than 4 loads per slot (the
//                                 staged-x wait then counts nothing)
#ifndef NF4_ABL_RING_FULL
#define NF4_ABL_RING_FULL 1
#endif
#ifndef NF4_ABL_ENTRY_RETURN  // tools: persistent kernel returns at entry (launch cost alone)
#define NF4_ABL_ENTRY_RETURN 0
#endif
#ifndef NF4_ABL_PLOAD_FAKE  // tools: persistent kernel's scale loads made from their offsets
#define NF4_ABL_PLOAD_FAKE 0
#endif
#ifndef NF4_PERSIST_PAIR  // persistent kernel: two ring slots decoded step-interleaved (even P)
#define NF4_PERSIST_PAIR 0
#endif
#ifndef NF4_ABL_LOOP_ON  // tools: persistent kernel skips its chunk loop (prologue + epilogue alone)
#define NF4_ABL_LOOP_ON 1
#endif
#ifndef NF4_ABL_KEEP_SLICE
#define NF4_ABL_KEEP_SLICE(ks_) true
#endif
#ifndef NF4_ABL_MMA_ON
#define NF4_ABL_MMA_ON 1
#define NF4_ABL_RED_ON 1
#define NF4_ABL_HANDOFF_ON 1
#endif

// Split-K hand-off, in the HIP memory model with relaxed agent-scope atomics
// only (no fence, no cache-policy assumption).  A slab entry is one 64-bit word
// holding the fp32 partials of two adjacent columns (c, c + 1; c even), each as
// the bitwise NOT of its bits: 0 = empty (the zero-filled workspace's state),
// both halves nonzero = written.  Each K slice issues its partials as atomic
// stores, then one lane draws a ticket on the strip's counter (atomic add; no wait
// for the stores to complete -- the ticket only elects the reducer); the
// slice drawing ksplit - 1 resets the counter and reduces: it reads every slice's
// entries with atomic loads, waiting per entry until it is written (per-location
// coherence: it sees the store once it is made; the entry held 0 since the
// previous call's reader cleared it, ordered by the kernel boundary), sums them
// in slice order (bitwise reproducible) and clears them for the next call.  The
// reader waits only on slices that already drew their tickets, i.e. are running
// or done, so the wait ends; it is bounded anyway: after kSpinMax polls the
// missing partials read as NaN AND the workspace's sticky error word (kErrWord,
// after the counters) is set, so the host learns of it (nf4_gemm_check_workspace)
// instead of finding NaNs nobody reported -- never a hung GPU, never a silent one.
// The word also poisons later calls on the same workspace: a slice that timed out
// may still store its partial after the reducer cleared the entry, and a later call
// would read that stale entry as written; so while the word is set every reducer
// writes NaN instead of its sum, until the host's check re-zeroes the workspace.
constexpr int kSpinMax = 1 << 16;
constexpr uint32_t kErrWord = 16384;  // uint32 index in the workspace header (byte 64 KiB)

// A partial's bits on the wire: its NOT, except that the one NaN whose NOT would be
// 0 (0xFFFFFFFF) goes as the NaN 0x7FFFFFFF -- so a written half is never 0 and a
// reader never mistakes a written entry for an empty one.
__device__ __forceinline__ uint32_t slab_not(float f) {
    const uint32_t b = __float_as_uint(f);
    return b == 0xFFFFFFFFu ? 0x80000000u : ~b;
}

__device__ __forceinline__ void slab_put2(uint64_t* slab, uint32_t e, float lo, float hi) {
    const uint64_t w = ((uint64_t)slab_not(hi) << 32) | (uint64_t)slab_not(lo);
    __hip_atomic_store(slab + e, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool slab_full(uint64_t w) { return (uint32_t)w != 0u && (uint32_t)(w >> 32) != 0u; }

// Entry of (slice ks, row m, column pair of c) in a slab of ncols columns.
__device__ __forceinline__ uint32_t slab_entry(uint32_t ks, uint32_t M, uint32_t m, uint32_t ncols, uint32_t c) {
    return (ks * M + m) * (ncols >> 1) + (c >> 1);
}

// One lane's partial of column `col`, where lanes l and l ^ 1 hold columns col and
// col ^ 1 of the same row: the even-column lane stores the pair.  All lanes call it.
__device__ __forceinline__ void slab_put_lane(uint64_t* slab, uint32_t e, float v, uint32_t col, bool valid) {
    const float nb = __shfl_xor(v, 1, 64);
    if (valid && !(col & 1u)) slab_put2(slab, e, v, nb);
}

// Poll the entries of v[][] that are not written yet, all of them per round (one
// memory round trip per round, not one per entry), at most kSpinMax rounds; an
// entry still empty then reads as the NOT of two NaNs and the lane sets the sticky
// error word *err (a reported wrong result, never a hung GPU).  Entries not to
// read are ~0 (full) on entry.
template <int KK, int KU>
__device__ __forceinline__ void splitk_poll(uint64_t* slab, uint32_t sstride, uint32_t k0, const uint32_t (&idx)[KU],
                                            uint64_t (&v)[KK][KU], uint32_t* err) {
    for (int tries = 0; tries < kSpinMax; ++tries) {
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int j = 0; j < KK; ++j)
#pragma unroll
            for (int u = 0; u < KU; ++u)
                if (!slab_full(v[j][u]))
                    v[j][u] = __hip_atomic_load(slab + (k0 + j) * sstride + idx[u], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int j = 0; j < KK; ++j)
#pragma unroll
            for (int u = 0; u < KU; ++u) ok = ok && slab_full(v[j][u]);
        if (__all(ok)) return;
    }
#pragma unroll
    for (int j = 0; j < KK; ++j)
#pragma unroll
        for (int u = 0; u < KU; ++u)
            if (!slab_full(v[j][u])) {
                v[j][u] = 0x803FFFFF803FFFFFull;  // NOT of two NaNs
                __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // vector atomic
            }
}

__device__ __forceinline__ bool splitk_ticket(uint32_t* ctr, uint32_t ksplit) {
    const uint32_t t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t != ksplit - 1u) return false;
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// The last arriver's split-K sum for one column group of KCOLS columns: slab
// [ksplit][M][ncols / 2] entries, columns col0.. -> y[m][ycol0 ..] (row stride yld).
// One wave; every lane owns kU entries (column pairs) of the group, and kU x kK
// loads are in flight before any wait -- they come from other XCDs' stores
// (L2-missing), so waiting per entry would serialise them.
template <int DT, uint32_t KCOLS>
__device__ __forceinline__ void splitk_reduce(uint64_t* slab, uint32_t ksplit, uint32_t M, uint32_t ncols,
                                              uint32_t col0, void* y, uint32_t yld, uint32_t ycol0, uint32_t lane,
                                              uint32_t* counters) {
    constexpr uint32_t KP = KCOLS / 2;  // entries per row of the group
    constexpr int kU = 4, kK = 4;
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    const uint32_t total = M * KP;
    const uint32_t sstride = M * (ncols >> 1);  // entries per slice
    // a workspace whose error word is set may hold stale entries: report, never sum them
    const bool poisoned = __hip_atomic_load(counters + kErrWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    for (uint32_t base = 0; base < total; base += 64u * kU) {
        float s0[kU], s1[kU];
        uint32_t idx[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t e = base + lane + 64u * u;
            idx[u] = e < total ? slab_entry(0, M, e / KP, ncols, col0 + 2u * (e % KP)) : kNone;
            s0[u] = s1[u] = 0.0f;
        }
        for (uint32_t k0 = 0; k0 < ksplit; k0 += kK) {
            uint64_t v[kK][kU];
            bool ok = true;
#pragma unroll
            for (int j = 0; j < kK; ++j)
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const bool live = k0 + j < ksplit && idx[u] != kNone;
                    v[j][u] = live ? __hip_atomic_load(slab + (k0 + j) * sstride + idx[u], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : ~0ull;
                    ok = ok && slab_full(v[j][u]);
                }
            if (!__all(ok)) splitk_poll<kK, kU>(slab, sstride, k0, idx, v, counters + kErrWord);  // not written yet
#pragma unroll
            for (int j = 0; j < kK; ++j) {
                if (k0 + j >= ksplit) break;  // uniform
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const float f0 = __uint_as_float(~(uint32_t)v[j][u]);
                    const float f1 = __uint_as_float(~(uint32_t)(v[j][u] >> 32));
                    s0[u] = (k0 + j == 0) ? f0 : s0[u] + f0;
                    s1[u] = (k0 + j == 0) ? f1 : s1[u] + f1;
                    if (idx[u] != kNone)  // empty again for the next call
                        __hip_atomic_store(slab + (k0 + j) * sstride + idx[u], 0ull, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t e = base + lane + 64u * u;
            if (e < total) {
                uint32_t* dst = reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(y) + (e / KP) * yld + ycol0 +
                                                            2u * (e % KP));
                *dst = poisoned ? pack2<DT>(__builtin_nanf(""), __builtin_nanf("")) : pack2<DT>(s0[u], s1[u]);
            }
        }
    }
}

// Two K slices: the hand-off by exchange, one memory round trip.  Both slices
// swap their pair of partials into the same slab entry (atomic exchange, relaxed,
// agent scope); exactly one of them gets back 0 (empty) and is done, the other
// gets back its partner's pair, sums the two in slice order (p0 + p1, bitwise the
// same as splitk_reduce), writes y and stores 0 so the entry is empty for the next
// call (ordered by the kernel boundary).  No ticket, no poll.  Partials go through
// slab_not as in slab_put2, so a written entry is never 0.
// Exchange entries are laid out [strip][row][column pair] (a strip's M x 8 pairs
// contiguous), so consecutive lanes of the exchange loops hit consecutive 8-byte
// entries: 512 contiguous bytes per wave instruction instead of 64-byte pieces of
// eight rows.  Same footprint as one slice of the [ks][M][ncols / 2] slab.
__device__ __forceinline__ uint32_t swap_entry(uint32_t strip, uint32_t M, uint32_t m, uint32_t col) {
    return (strip * M + m) * 8u + (col >> 1);
}
__device__ __forceinline__ uint64_t slab_swap2(uint64_t* p, float lo, float hi) {
    const uint64_t w = ((uint64_t)slab_not(hi) << 32) | (uint64_t)slab_not(lo);
    return __hip_atomic_exchange(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int DT>
__device__ __forceinline__ void store_y(void* y, uint32_t i, float v) {
    if constexpr (DT == NF4DQ_BF16) {
        reinterpret_cast<__bf16*>(y)[i] = (__bf16)v;
    } else {
        reinterpret_cast<_Float16*>(y)[i] = (_Float16)opaque(v);
    }
}
constexpr uint32_t kChunkK = 128;

// One weight of a 128-deep launch; weights that share x (q/k/v, gate/up) go in
// one launch, column groups numbered over all of them.
constexpr int kK128GroupMax = 8;
struct K128Mat {
    const uint8_t* packed;  // [N][K/2]
    const uint8_t* a1;      // [nb]
    const float* a2;        // [n2]
    void* y;                // [M][N] fp16/bf16
    uint32_t N;
    uint32_t cg_begin;      // first column group of this weight in the launch
    uint32_t col_begin;     // first column in the launch (split-K slab column)
    FastDiv nb, n2;
};

struct GemmArgs {
    K128Mat mat[kK128GroupMax];
    uint32_t nmat;
    const void* x;          // [M][K] fp16/bf16
    uint64_t* slab;         // [ksplit][M][ncols] tagged fp32 partials (ksplit > 1; splitk_reduce)
    uint32_t* counters;     // one split-K ticket per column group, 0 between calls
    uint32_t M, K;
    uint32_t ncols;         // sum of N
    uint32_t col_groups;    // column groups (16 NT columns) over all weights
    uint32_t ksplit;
    uint32_t chunks_per_split;
    uint32_t chunks;        // K / 128
    uint32_t bpr, groups;   // K / 64, ceil(bpr / 4)
    uint32_t per_wg;        // register-resident kernel: strips per workgroup
};

// One 128-deep K chunk of one lane: for each of the wave's NT 16-column strips,
// 16 packed weight bytes of its row there (one 64-block, so one scale), and
// MT x 4 activation fragments -- shared by the NT strips, so a wider wave
// (NT > 1) loads x once per NT weights instead of once per weight.
template <int MT, int NT>
struct Chunk {
    u32x4 w[NT];
    uint32_t qa[NT];    // absmax bytes
    float qb[NT];       // nested absmax
    u32x4 x[MT][4];
};

// VS: the block scales come from the workgroup's LDS table (nf4_gemm_smallm_kernel), no per-chunk gathers
template <int MT, int NT, bool VS>
__device__ __forceinline__ void chunk_issue(const GemmArgs& A, const K128Mat& Mt, __amdgpu_buffer_rsrc_t rw,
                                            __amdgpu_buffer_rsrc_t rx, uint32_t c, bool valid, uint32_t row,
                                            uint32_t nl, uint32_t kh, Chunk<MT, NT>& in) {
    const uint32_t kbase = c * kChunkK + 32u * kh;
    // past the wave's last chunk: offsets beyond the buffer ranges (zeros, no traffic)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
        in.w[nt] = __builtin_amdgcn_raw_buffer_load_b128(
            rw, valid ? (row + 16u * nt) * (A.K >> 1) + (kbase >> 1) : 0xFFFFFFF0u, 0, 0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const uint32_t xoff = valid ? ((16u * mt + nl) * A.K + kbase) * 2u : 0xFFFFFF00u;  // rows >= M: zeros
#pragma unroll
        for (int s = 0; s < 4; ++s) in.x[mt][s] = __builtin_amdgcn_raw_buffer_load_b128(rx, xoff + 16u * s, 0, 0);
    }
    if constexpr (!VS) {
        const uint32_t b = 2u * (valid ? c : 0u) + (kh >> 1);  // 64-block within the row
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const uint32_t r = row + 16u * nt;
            in.qa[nt] = Mt.a1[fmodu(r * A.bpr + b, Mt.nb)];             // (:173-177 wrap)
            in.qb[nt] = Mt.a2[fmodu(r * A.groups + (b >> 2), Mt.n2)];  // (:40-41, :183-186 wrap)
        }
    }
}

template <int DT, int MT, int NT>
__device__ __forceinline__ void chunk_mma(const Chunk<MT, NT>& in, const float* lut, const float (&scs)[NT],
                                          f32x4 (&acc)[MT][NT]) {
    const char* t = reinterpret_cast<const char*>(lut);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const float sc = scs[nt];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint32_t wd = in.w[nt][s];
            const uint32_t hi4 = (wd >> 2) & 0x3C3C3C3Cu;
            const uint32_t lo4 = (wd << 2) & 0x3C3C3C3Cu;
            float v[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[2 * k] = *reinterpret_cast<const float*>(t + ((hi4 >> (8 * k)) & 0xFFu)) * sc;
                v[2 * k + 1] = *reinterpret_cast<const float*>(t + ((lo4 >> (8 * k)) & 0xFFu)) * sc;
            }
            // the exact weights nf4_dequant_ref writes: fp32 product, RNE to 16 bits
            const u32x4 bw = {pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]),
                              pack2<DT>(v[6], v[7])};
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                if constexpr (DT == NF4DQ_BF16) {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, in.x[mt][s]), __builtin_bit_cast(bf16x8, bw), acc[mt][nt], 0, 0, 0);
                } else {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                        __builtin_bit_cast(f16x8, in.x[mt][s]), __builtin_bit_cast(f16x8, bw), acc[mt][nt], 0, 0, 0);
                }
            }
        }
    }
}

// Workgroup = WV waves owning 16 NT output columns (NT strips) of one K slice;
// wave w takes every WV-th group of D chunks, D chunks in flight at a time; the
// waves' partial sums are combined through LDS (fixed order, one strip at a time).
template <int DT, int MT, int D, int WV, int NT, bool VS>
__global__ __launch_bounds__(64 * WV) void nf4_gemm_smallm_kernel(const GemmArgs A) {
    constexpr int kGemmWaves = WV;
    __shared__ __attribute__((aligned(16))) float lut[20];  // 16 codes + the last-arriver flag
    __shared__ __attribute__((aligned(16))) f32x4 red[WV][MT][64];
    extern __shared__ __attribute__((aligned(16))) float scl[];  // VS: [16 NT rows][2 chunks_per_split blocks]
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t nl = lane & 15u, kh = lane >> 4;
    const uint32_t cg = blockIdx.x % A.col_groups;   // group of NT 16-column strips, launch-wide
    const uint32_t ks = blockIdx.x / A.col_groups;   // K slice
    uint32_t mi = 0;                                 // the weight this workgroup works on (uniform scan)
    for (uint32_t i = 1; i < A.nmat; ++i) mi = cg >= A.mat[i].cg_begin ? i : mi;
    const K128Mat& Mt = A.mat[mi];
    const uint32_t cgl = cg - Mt.cg_begin;           // group within the weight
    const uint32_t row = cgl * 16u * NT + nl;        // this lane's row in strip 0; strip nt adds 16 nt
    // a slice may start past the end (e.g. K = 4096, ksplit = 12: ceil(32/12) = 3
    // chunks per slice, slice 11 starts at 33): clamp so it is empty (c1 == c0),
    // never a wrapped block count
    const uint32_t c0s = ks * A.chunks_per_split;
    const uint32_t c0 = c0s < A.chunks ? c0s : A.chunks;
    const uint32_t c1 = c0 + A.chunks_per_split < A.chunks ? c0 + A.chunks_per_split : A.chunks;

    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.packed, 0, Mt.N * (A.K >> 1), kRsrcFlags);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, 0, A.M * A.K * 2u, kRsrcFlags);

    f32x4 acc[MT][NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint32_t nbs = 2u * A.chunks_per_split;  // VS: scale blocks per row in the table
    bool first = true;
    for (uint32_t g = c0 + wave * D; g < c1 || first; g += kGemmWaves * D) {
        Chunk<MT, NT> ch[D];
#pragma unroll
        for (int d = 0; d < D; ++d) chunk_issue<MT, NT, VS>(A, Mt, rw, rx, g + d, g + d < c1, row, nl, kh, ch[d]);
        if (first) {  // LUT (+ VS: the slice's scale table) and the barrier overlap the first loads
            write_lut(lut);
            if constexpr (VS) {
                // the workgroup's 16 NT rows x this slice's blocks: coalesced byte / float
                // loads (consecutive threads, consecutive blocks of a row), one IEEE
                // division per block (:45), instead of per-lane gathers in every chunk
                const uint32_t r0 = cgl * 16u * NT, b0 = 2u * c0, nbl = 2u * (c1 - c0);
                for (uint32_t i = threadIdx.x; i < 16u * NT * nbs; i += 64u * WV) {
                    const uint32_t rr = i / nbs, j = i - rr * nbs;
                    if (j < nbl) {
                        const uint32_t r = r0 + rr, gb = b0 + j;  // no wrap inside a row (host-checked)
                        const float q = (float)Mt.a1[fmodu(r * A.bpr, Mt.nb) + gb];
                        scl[i] = (q / 127.0f) * Mt.a2[fmodu(r * A.groups, Mt.n2) + (gb >> 2)];
                    }
                }
            }
            __syncthreads();
            first = false;
        }
#pragma unroll
        for (int d = 0; d < D; ++d) {
            float scs[NT];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                if constexpr (VS) {
                    const uint32_t j = 2u * (g + d - c0) + (kh >> 1);
                    scs[nt] = g + d < c1 ? scl[(16u * nt + nl) * nbs + j] : 0.0f;
                } else {
                    scs[nt] = ((float)ch[d].qa[nt] / 127.0f) * ch[d].qb[nt];  // IEEE division, fp32 multiply (:45)
                }
            }
            chunk_mma<DT, MT, NT>(ch[d], lut, scs, acc);
        }
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        if (nt) __syncthreads();  // wave 0 has read the previous strip's partials
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) red[wave][mt][lane] = acc[mt][nt];
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                f32x4 s = red[0][mt][lane];
#pragma unroll
                for (int w = 1; w < kGemmWaves; ++w) s += red[w][mt][lane];
                acc[mt][nt] = s;
            }
        }
    }
    if (wave != 0) return;

    // acc[mt][nt][r] = Y[16 mt + 4 kh + r][row + 16 nt]
    if (A.ksplit == 1) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t m = 16u * mt + 4u * kh + r;
                    if (m < A.M) store_y<DT>(Mt.y, m * Mt.N + row + 16u * nt, acc[mt][nt][r]);
                }
            }
        return;
    }

    // Split-K, reduced inside the launch: every slice writes its fp32 partials,
    // drains them, and one lane takes a ticket on the column group's counter
    // (splitk_ticket / splitk_reduce); the workgroup drawing ksplit-1 sums all
    // slices in slice order and writes y.  Bitwise reproducible.
    const uint32_t scol = Mt.col_begin + row;  // slab column of this lane (strip 0)
    if (NF4_ABL_KEEP_SLICE(ks))
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t m = 16u * mt + 4u * kh + r;
                slab_put_lane(A.slab, slab_entry(ks, A.M, m, A.ncols, scol + 16u * nt), acc[mt][nt][r], scol, m < A.M);
            }
        }
    uint32_t last = 0;
    if (lane == 0) last = splitk_ticket(&A.counters[cg], A.ksplit);
    last = __builtin_amdgcn_readfirstlane(last);
    if (!last) return;
    splitk_reduce<DT, 16u * NT>(A.slab, A.ksplit, A.M, A.ncols, Mt.col_begin + cgl * 16u * NT, Mt.y, Mt.N,
                                cgl * 16u * NT, lane, A.counters);
}

// ---------------------------------------------------------------------------
// Shared-activation decode kernel (K % 128 == 0; built for 16 < M <= 32).  The
// 128-deep kernel's waves split K over the same columns, so every workgroup
// streams the whole x[M][K] through its vector-memory path and a wave can hold
// only one or two weight chunks in registers next to its x fragments -- at
// M = 32 that left 7 waves per CU with ~28 KB of weight bytes in flight and the
// address FIFO saturated (profiles/r01/pmc_gemm_m32_14336x4096.txt).  Here a
// workgroup owns WV 16-column strips (one per wave) over one K slice of KC
// 128-deep chunks:
//  * the slice of x (M x KC*128 bf16, rows padded 16 B so consecutive rows
//    start 4 banks apart) is loaded ONCE per workgroup and read by all WV
//    waves from LDS (ds_read_b128), so x costs 1/WV of the vector-memory
//    instructions and no registers between chunks;
//  * each wave issues ALL KC of its weight chunks (16 B per lane each) before
//    it waits on anything, so a CU with two workgroups of 8 waves keeps
//    16 x KC KiB of weight bytes in flight;
//  * the block scales of the workgroup's 16 WV rows x 2 KC blocks are built once
//    in LDS from gathers with the reference's wrap (any nb / n2);
//  * K slices over workgroups meet in the fp32 slab: one ticket per strip, the
//    last arriver sums the slices in slice order (bitwise reproducible).
// Same k permutation, dequant and MFMA step as the 128-deep kernel (chunk_mma).
template <int DT, int MT, int KC, int WV>
__global__ __launch_bounds__(64 * WV, 4) void nf4_gemm_xs_kernel(const GemmArgs A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr uint32_t XS = KC * 256u + 16u;                 // LDS bytes per staged x row
    constexpr uint32_t kScl = 16u * MT * XS;                 // scale table [16 WV rows][2 KC blocks]
    constexpr uint32_t kLut = kScl + 16u * WV * 2u * KC * 4u;
    float* scl = reinterpret_cast<float*>(smem + kScl);
    float* lut = reinterpret_cast<float*>(smem + kLut);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t nl = lane & 15u, kh = lane >> 4;
    const uint32_t cg = blockIdx.x % A.col_groups;  // group of WV strips, launch-wide
    const uint32_t ks = blockIdx.x / A.col_groups;  // K slice
    uint32_t mi = 0;                                // the weight this workgroup works on (uniform scan)
    for (uint32_t i = 1; i < A.nmat; ++i) mi = cg >= A.mat[i].cg_begin ? i : mi;
    const K128Mat& Mt = A.mat[mi];
    const uint32_t strip0 = (cg - Mt.cg_begin) * (uint32_t)WV;  // first strip of this workgroup in the weight
    const uint32_t strip = strip0 + wave;
    const bool live = strip < (Mt.N >> 4);          // wave-uniform (a weight's last group may be partial)
    const uint32_t row = strip * 16u + nl;
    const uint32_t c0s = ks * (uint32_t)KC;
    const uint32_t c0 = c0s < A.chunks ? c0s : A.chunks;  // an empty last slice: c1 == c0
    const uint32_t c1 = c0 + KC < A.chunks ? c0 + KC : A.chunks;
    const uint32_t kc = c1 - c0;

    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.packed, 0, Mt.N * (A.K >> 1), kRsrcFlags);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, 0, A.M * A.K * 2u, kRsrcFlags);

    // 1. the x slice (rows >= M and chunks past c1 read as zeros: out-of-range offsets)
    constexpr uint32_t kPpr = KC * 16u;              // 16-byte pieces per row
    constexpr uint32_t kPieces = 16u * MT * kPpr;
    constexpr int XR = (int)((kPieces + 64u * WV - 1u) / (64u * WV));
    u32x4 xv[XR];
#pragma unroll
    for (int i = 0; i < XR; ++i) {
        const uint32_t p = tid + (uint32_t)i * 64u * WV;
        const uint32_t r = p / kPpr, q = p % kPpr;
        const bool ok = p < kPieces && r < A.M && q < kc * 16u;
        xv[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? (r * A.K + c0 * kChunkK) * 2u + q * 16u : kOob, 0, 0);
    }
    // 2. the block-scale gathers of the workgroup's rows (reference wrap, :173-186)
    constexpr uint32_t kSclN = 16u * WV * 2u * KC;
    constexpr int SR = (int)((kSclN + 64u * WV - 1u) / (64u * WV));
    uint32_t qa[SR];
    float qb[SR];
#pragma unroll
    for (int i = 0; i < SR; ++i) {
        const uint32_t e = tid + (uint32_t)i * 64u * WV;
        const uint32_t rr = e / (2u * KC), j = e % (2u * KC);
        const uint32_t r = strip0 * 16u + rr, b = 2u * c0 + j;
        const bool ok = e < kSclN && r < Mt.N && j < 2u * kc;
        qa[i] = ok ? Mt.a1[fmodu(r * A.bpr + b, Mt.nb)] : 0u;
        qb[i] = ok ? Mt.a2[fmodu(r * A.groups + (b >> 2), Mt.n2)] : 0.0f;
    }
    // 3. every weight chunk of this wave, all in flight before the first wait
    u32x4 w[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        const uint32_t c = c0 + (uint32_t)j;
        w[j] = __builtin_amdgcn_raw_buffer_load_b128(
            rw, live && (uint32_t)j < kc ? row * (A.K >> 1) + ((c * kChunkK + 32u * kh) >> 1) : kOob, 0, 0);
    }
    // 4. tables and the staged slice (waits for x and the scale gathers only), one barrier
    write_lut(lut);
#pragma unroll
    for (int i = 0; i < SR; ++i) {
        const uint32_t e = tid + (uint32_t)i * 64u * WV;
        if (e < kSclN) scl[e] = ((float)qa[i] / 127.0f) * qb[i];  // IEEE division, fp32 multiply (:45)
    }
#pragma unroll
    for (int i = 0; i < XR; ++i) {
        const uint32_t p = tid + (uint32_t)i * 64u * WV;
        if (p < kPieces) *reinterpret_cast<u32x4*>(smem + (p / kPpr) * XS + (p % kPpr) * 16u) = xv[i];
    }
    __syncthreads();

    // 5. the chunks: x fragments from LDS, the wave's weights from registers
    f32x4 acc[MT][1];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint32_t srow = (wave * 16u + nl) * 2u * KC + (kh >> 1);
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        if ((uint32_t)j < kc) {  // uniform
            Chunk<MT, 1> ch;
            ch.w[0] = w[j];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    ch.x[mt][s] = *reinterpret_cast<const u32x4*>(smem + (16u * mt + nl) * XS + (uint32_t)j * 256u +
                                                                 64u * kh + 16u * s);
            const float scs[1] = {scl[srow + 2u * (uint32_t)j]};
            chunk_mma<DT, MT, 1>(ch, lut, scs, acc);
        }
    }
    if (!live) return;

    // acc[mt][0][r] = Y[16 mt + 4 kh + r][row]
    if (A.ksplit == 1) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t m = 16u * mt + 4u * kh + r;
                if (m < A.M) store_y<DT>(Mt.y, m * Mt.N + row, acc[mt][0][r]);
            }
        return;
    }
    // split-K: this wave's strip slice to the slab; one ticket per strip; the last
    // arriver sums the slices in slice order (splitk_ticket / splitk_reduce)
    const uint32_t scol = Mt.col_begin + row;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t m = 16u * mt + 4u * kh + r;
            slab_put_lane(A.slab, slab_entry(ks, A.M, m, A.ncols, scol), acc[mt][0][r], scol, m < A.M);
        }
    const uint32_t ctr = (Mt.col_begin >> 4) + strip;
    uint32_t last = 0;
    if (lane == 0) last = splitk_ticket(&A.counters[ctr], A.ksplit);
    last = __builtin_amdgcn_readfirstlane(last);
    if (!last) return;
    splitk_reduce<DT, 16u>(A.slab, A.ksplit, A.M, A.ncols, Mt.col_begin + strip * 16u, Mt.y, Mt.N, strip * 16u, lane, A.counters);
}

// ---------------------------------------------------------------------------
// Register-resident activation kernel (NF4DQ_GEMM_XR; K % 128 == 0, any M <= 32).
// The kernels above re-read x for every column strip they take (from L2 or from
// an LDS slice staged per workgroup), and cover K with many small slices, so
// every launch pays a per-workgroup prologue and a wide split-K hand-off.  Here
// the K split is over the WAVES of one workgroup instead:
//  * wave w of K slice ks owns KPW 128-deep chunks, (ks * WV + w) * KPW ..; it
//    loads its x fragments for them ONCE, into registers (MT x 4 x KPW 16-byte
//    loads per lane), and keeps them for the whole launch;
//  * the workgroup walks its T column strips (16 columns each, numbered over all
//    the weights of the launch): per strip a wave needs KPW 16-byte weight loads
//    per lane plus its scale gathers (reference wrap), held in a D-deep register
//    ring refilled as each strip is consumed;
//  * the WV partial 16-column tiles of a strip meet in LDS (double-buffered, one
//    barrier per strip); one wave per 16-row tile sums them in wave order and
//    keeps the fp32 result in LDS until the loop ends (no global store among the
//    ring's loads, so no wait drains the ring);
//  * WV * KPW * 128 = K needs no split across workgroups (M <= 16, K = 4096:
//    16 waves x 2 chunks); otherwise ksplit = ceil(K / 128 / (WV * KPW)) slices
//    meet in the fp32 slab with one ticket per strip, summed in slice order.
// Same k permutation, dequant and MFMA step as the 128-deep kernel (chunk_mma),
// so the weights entering the MFMAs are exactly nf4_dequant_ref's.
// KPW = 1: one 128-deep chunk per wave (lane: 16 B of its row); KPW = 2: one
// 256-deep chunk (lane: 32 contiguous bytes = one 64-block, so a wave's loads
// cover whole 128-byte lines of its 16 rows, and one scale per lane); KPW = 4:
// two consecutive 256-deep chunks (8 waves then span K = 4096 without a K split).
template <int KPW>
struct XSlot {
    static constexpr int NSC = KPW == 4 ? 2 : 1;  // 64-blocks (scales) per lane: one per 256-deep sub-chunk
    u32x4 w[KPW];
    uint8_t qa[NSC];  // kept 8-bit: a widening right after the load would wait for it (a drained ring)
    float qb[NSC];
};

// The weight owning a strip: straight-line selects over the group (no loop in
// the strip loop -- a loop there costs the ring its counted waits)
__device__ __forceinline__ uint32_t xr_mat_of(const GemmArgs& A, uint32_t strip) {
    uint32_t mi = 0;
#pragma unroll
    for (int i = 1; i < kK128GroupMax; ++i) mi = (uint32_t)i < A.nmat && strip >= A.mat[i].cg_begin ? (uint32_t)i : mi;
    return mi;
}

// Lane-constant parts of a strip's offsets (computed once): every per-strip term
// is then a scalar plus this -- no per-strip vector multiply-add, whose 64-bit
// form reads an unrelated (possibly still loading) register half and turns the
// ring's counted waits into drains.
struct XLane {
    uint32_t w;   // the lane's bytes within a 16-row chunk: nl K/2 + 16 kh (KPW 1) / 32 kh (KPW 2)
    uint32_t b1;  // the lane's 64-block within the strip's rows: nl bpr + kh/2 (KPW 1) / kh (KPW 2)
    uint32_t b2;  // nl * groups
};

// The weight the ring is issuing from, kept in scalar registers: the strips of a
// workgroup rarely cross into the next weight of a group, so the descriptor loads
// (scalar memory, waited for before the refill's first vector load) happen once per
// weight, not once per strip.
struct XMat {
    __amdgpu_buffer_rsrc_t rw, ra1, ra2;
    FastDiv nb, n2;
    uint32_t begin, next;  // [begin, next): the cached weight's strips in the launch
};

__device__ __forceinline__ void xmat_load(const GemmArgs& A, uint32_t strip, XMat& m) {
    const uint32_t mi = xr_mat_of(A, strip);
    const K128Mat& Mt = A.mat[mi];
    m.rw = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.packed, 0, Mt.N * (A.K >> 1), kRsrcFlags);
    m.ra1 = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.a1, 0, Mt.nb.d, kRsrcFlags);
    m.ra2 = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.a2, 0, Mt.n2.d * 4u, kRsrcFlags);
    m.nb = Mt.nb;
    m.n2 = Mt.n2;
    m.begin = Mt.cg_begin;
    m.next = mi + 1u < A.nmat ? A.mat[mi + 1u].cg_begin : 0xFFFFFFFFu;
}

template <int KPW>
__device__ __forceinline__ void xslot_issue(const GemmArgs& A, uint32_t strip, bool valid, uint32_t cw,
                                            const XLane& ln, XMat& Mt, XSlot<KPW>& s) {
    if (strip >= Mt.next) xmat_load(A, strip, Mt);  // uniform; scalar loads only
    const uint32_t r0 = (strip - Mt.begin) * 16u;  // first row of the strip (uniform)
    const __amdgpu_buffer_rsrc_t rw = Mt.rw, ra1 = Mt.ra1, ra2 = Mt.ra2;
    constexpr int NSC = XSlot<KPW>::NSC;
#pragma unroll
    for (int h = 0; h < NSC; ++h) {
        const uint32_t c = cw + 2u * (uint32_t)h;  // first 128-deep chunk of this sub-chunk
        // invalid (past the strips or past K): offsets beyond every range -- zeros, no
        // traffic, and still one counted load each (a straight-line ring)
        const uint32_t oob = valid && c + (KPW == 1 ? 0u : 1u) < A.chunks ? 0u : kOob;
        // the lane's block: 2c + kh/2 (KPW 1) / 4 (c/2) + kh = 2c + kh (256-deep); its
        // nested group (block / 4) is c / 2 either way (uniform)
        const uint32_t w0 = r0 * (A.K >> 1) + c * 64u + ln.w;
        constexpr int WQ = KPW == 1 ? 1 : 2;  // 16-byte weight loads per sub-chunk
#pragma unroll
        for (int q = 0; q < WQ; ++q)
            s.w[WQ * h + q] = NF4_ABL_WLOAD(rw, (w0 + 16u * q) | oob);
        s.qa[h] = (uint8_t)NF4_ABL_SLOAD(ra1, fmodu(r0 * A.bpr + 2u * c + ln.b1, Mt.nb) | oob, true);  // (:173-177)
        s.qb[h] = __uint_as_float(
            NF4_ABL_SLOAD(ra2, (fmodu(r0 * A.groups + (c >> 1) + ln.b2, Mt.n2) * 4u) | oob, false));  // (:40-41, :183-186)
    }
}

// Dequant + MFMA of one 256-deep chunk with the activations in registers (KPW = 2):
// the streaming kernel's pair-table lookups (sslot_mma: one conflict-free
// ds_read_b64 per packed byte = two weights, issued LA steps ahead), the fp32
// products with the block scale, one RNE pack per pair; x fragment (q, s) of step
// st = 4 q + s carries the same k as weight dword st (same permutation).
template <int DT, int MT>
__device__ __forceinline__ void xr_pair_mma(const u32x4& w0, const u32x4& w1, float sc, const f32x2* ptab,
                                            uint32_t slot8, const u32x4 (&xf)[2][MT][4], f32x4 (&acc)[MT]) {
    const f32x2 sc2 = {sc, opaque(sc)};
    const char* pt = reinterpret_cast<const char*>(ptab);
    // MT = 2 holds 64 VGPRs of x: a shorter lookahead, and its two row tiles already
    // give two independent MFMA chains (no second accumulator set)
    constexpr int LA = MT == 2 ? 2 : 3;
    f32x2 v[8][4];
    f32x4 accb[MT == 2 ? 1 : MT];
#pragma unroll
    for (int mt = 0; mt < (MT == 2 ? 1 : MT); ++mt) accb[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto issue = [&](int st) {
        const uint32_t wd = st < 4 ? w0[st] : w1[st - 4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t addr = __builtin_amdgcn_perm(wd, slot8, 0x0C0C0000u | ((4u + b) << 8));
            v[st][b] = NF4_ABL_LOOKUP(pt, addr, wd);
        }
    };
#pragma unroll
    for (int st = 0; st < LA; ++st) issue(st);
#pragma unroll
    for (int st = 0; st < 8; ++st) {
        if (st + LA < 8) issue(st + LA);
        // (Round 2 had a scheduling barrier here after wrong strips were seen beyond a
        // workgroup's first.  Its stated cause -- scalar loads completing out of order
        // under counted LDS waits -- is not in the ISA: a scan of every s_waitcnt of
        // this kernel, at the commit that added the barrier and now, with and without
        // it, finds no counted lgkmcnt wait while a scalar load is outstanding.  Without
        // it the current kernel passes tools/xr_probe.py (58 configurations, 41 with
        // several strips per workgroup) and the GEMM suite, and is 0.1-0.4 us faster
        // per launch (profiles/r03/gemm/xr_no_sched_barrier.jsonl);
        // test_xr_multi_strip_workgroups keeps several strips per workgroup under test
        // at any CU count.)
        uint32_t bw[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const f32x2 p = v[st][b] * sc2;  // fp32 products (:97-98)
            bw[b] = pack2<DT>(p.x, p.y);     // RNE (:109-110)
        }
        const u32x4 bq = {bw[0], bw[1], bw[2], bw[3]};
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            f32x4& c = (MT == 1 && (st & 1)) ? accb[0] : acc[mt];
            const u32x4 a = xf[st >> 2][mt][st & 3];
            if constexpr (!NF4_ABL_MMA_ON) {
                asm volatile("" ::"v"(a), "v"(bq));
            } else if constexpr (DT == NF4DQ_BF16) {
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, bq),
                                                            c, 0, 0, 0);
            } else {
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, bq),
                                                           c, 0, 0, 0);
            }
        }
    }
    if constexpr (MT == 1) acc[0] += accb[0];
}

// Piece swizzle of the staged x rows (16-byte pieces 0..31 of a row's 512 bytes):
// piece c of local row r sits at slot c ^ xr_xsw(r).  In each ds_read_b128 lane
// group ({0-3,12-15,20-27}, ...: rows 0-3 and 12-15 of one 128-byte segment, rows
// 4-11 of the next) the 16 lanes then hit 16 distinct 4-bank sets.
__device__ __forceinline__ uint32_t xr_xsw(uint32_t r) { return r ^ ((((r + 4u) >> 3) & 1u) << 3); }

template <int DT, int MT, int WV, int KPW, int D, int GU>
__device__ __forceinline__ void xr_body(const GemmArgs& A) {
    extern __shared__ __attribute__((aligned(16))) f32x4 xr_smem[];  // dynamic part (host: xr_lds_dynamic)
    // 256-deep chunks: the pair table (64 KiB) and the q/127 table, static so that the
    // lookups' addresses need no base added (one VALU per two weights less than in a
    // dynamic region, whose base the compiler adds as a late-resolved 0)
    __shared__ __attribute__((aligned(16))) f32x2 xr_ptab[KPW >= 2 ? 256 * 32 : 2];
    __shared__ float xr_qtab[KPW >= 2 ? 256 : 4];
    f32x2* ptab = xr_ptab;
    float* qtab = xr_qtab;
    // partial tiles meet once per R strips (8 waves: two strips per barrier)
    constexpr int R = WV == 8 && D % 2 == 0 ? 2 : 1;
    static_assert(GU == 0 || (R * MT <= WV && D == R), "unrolled groups: one tile per wave and group");
    f32x4* red = xr_smem;                                    // [2][R][WV][MT][64] partial tiles
    float* lut = reinterpret_cast<float*>(red + 2 * R * WV * MT * 64);  // 16 codes
    uint32_t* last_flags = reinterpret_cast<uint32_t*>(lut + 16);        // [64] split-K tickets drawn last
    float* held = reinterpret_cast<float*>(last_flags + 64);            // [T][16 MT][16] fp32 results
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t nl = lane & 15u, kh = lane >> 4;
    const uint32_t S = A.ksplit, T = A.per_wg;
    const uint32_t ks = blockIdx.x % S;                      // K slice
    const uint32_t s0 = (blockIdx.x / S) * T;                // first strip (launch-wide)
    const uint32_t s1 = s0 + T < A.col_groups ? s0 + T : A.col_groups;
    const uint32_t nst = s1 > s0 ? s1 - s0 : 0u;
    const uint32_t cw = (ks * (uint32_t)WV + wave) * (uint32_t)KPW;  // the wave's first chunk
    const XLane ln{nl * (A.K >> 1) + (KPW >= 2 ? 32u : 16u) * kh, nl * A.bpr + (KPW >= 2 ? kh : kh >> 1),
                   nl * A.groups};
    NF4_GSTAMP_INIT(WV);
    NF4_GSTAMP(0);

    // 1. the wave's x fragments (rows >= M and chunks past K read as zeros),
    //    then the ring's first D strips, then the code table.  (Ring first measured
    //    slower: 21.9 vs 20.3 us at M = 32 on 14336x4096, profiles/r03/gemm.)
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, 0, A.M * A.K * 2u, kRsrcFlags);
    u32x4 xf[KPW][MT][4];
    // Staged form (one 256-deep chunk, two row tiles, 8 waves): a lane's fragments are
    // 128 contiguous bytes of one row, so a direct 16-byte load instruction touches 64
    // lines (16 rows x 4 lanes) and the wave's 16 of them queue behind each other in
    // the address path (the x issue was ~4.4 us of the prologue at M = 32,
    // profiles/r03/gemm).  Instead each LDS-DMA instruction reads two rows' 512 bytes
    // = 8 whole lines into the wave's own 8 KiB of LDS (row tile 0 in the reduction
    // buffer, row tile 1 in the pair table's region, both free until the tables are
    // written), and the fragments are read back with ds_read_b128.  Pieces are
    // swizzled within a row (piece c at slot c ^ xr_xsw(row)) so the reads are
    // conflict-free in every 16-lane group.
    constexpr bool kStage = KPW == 2 && MT == 2 && R == 2;
    const bool xlive = cw + (KPW == 1 ? 0u : 1u) < A.chunks;  // uniform: the wave's chunk inside K
    if constexpr (kStage) {
        if (xlive && NF4_ABL_X_ON) {
            const uint32_t rl = lane >> 5, slot = lane & 31u;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                char* reg = reinterpret_cast<char*>(mt == 0 ? (void*)red : (void*)xr_ptab) + wave * 8192u;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t r = 16u * mt + 2u * i + rl;  // row of this lane's piece
                    const uint32_t voff =
                        r < A.M ? (r * A.K + cw * kChunkK) * 2u + 16u * (slot ^ xr_xsw(2u * i + rl)) : kOob;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rx, (__attribute__((address_space(3))) void*)(reg + 1024 * i), 16, voff, 0, 0, 0);
                }
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < KPW; ++q)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                // k of fragment (q, s): 128 cw + 32 kh + 8 s (KPW 1), 128 cw + 256 (q / 2) + 64 kh
                // + 32 (q % 2) + 8 s (256-deep sub-chunks) -- the weight dword's k (same permutation)
                const uint32_t r = 16u * mt + nl;
                const uint32_t c = cw + (KPW == 1 ? 0u : 2u * (uint32_t)(q / 2));
                const uint32_t xoff = r < A.M && c + (KPW == 1 ? 0u : 1u) < A.chunks
                                          ? (r * A.K + c * kChunkK + (KPW == 1 ? 32u : 64u) * kh + 32u * (q % 2)) * 2u
                                          : kOob;
#pragma unroll
                for (int s = 0; s < 4; ++s) xf[q][mt][s] = __builtin_amdgcn_raw_buffer_load_b128(rx, xoff + 16u * s, 0, 0);
            }
    }
    __builtin_amdgcn_sched_barrier(0);  // issue order = wait order: x, then the ring slot by slot
    NF4_GSTAMP(11);
    XSlot<KPW> ring[D];
    XMat xm;
    xmat_load(A, s0, xm);
#pragma unroll
    for (int d = 0; d < D; ++d) {
        xslot_issue<KPW>(A, s0 + (uint32_t)d, (uint32_t)d < nst, cw, ln, xm, ring[d]);
        __builtin_amdgcn_sched_barrier(0);
    }
    NF4_GSTAMP(10);
    if constexpr (kStage) {
        // the x DMA went out before the ring's D x 4 loads: wait for it alone (the
        // compiler does not order LDS-DMA writes before these LDS reads by itself);
        // an ablation build whose ring issues fewer loads waits for everything
        if constexpr (NF4_ABL_RING_FULL) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * D) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // fragment (q, s) of row tile mt = piece 8 kh + 4 q + s of row 16 mt + nl
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const char* reg = reinterpret_cast<const char*>(mt == 0 ? (void*)red : (void*)xr_ptab) + wave * 8192u;
            const bool rok = xlive && 16u * mt + nl < A.M;
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(reg + nl * 512u + 16u * ((8u * kh + p) ^ xr_xsw(nl)));
                xf[p >> 2][mt][p & 3] = rok ? v : u32x4{0u, 0u, 0u, 0u};
            }
        }
        __syncthreads();  // every wave's fragments out of the pair table's region before the tables
    }
    write_lut(lut);
    if constexpr (KPW >= 2) {  // tables while the loads fly (as the streaming kernels)
        if (tid < 256u) qtab[tid] = (float)tid / 127.0f;  // IEEE division (:45)
        for (uint32_t u = tid; u < 16u * 32u; u += 64u * WV) {
            const float clo = nf4_code(u >> 5);
#pragma unroll
            for (int hi = 0; hi < 16; ++hi) ptab[(16u * hi + (u >> 5)) * 32u + (u & 31u)] = f32x2{nf4_code(hi), clo};
        }
    }
    const uint32_t slot8 = (lane & 31u) * 8u;
    NF4_GSTAMP(12);
    __syncthreads();
    NF4_GSTAMP(1);

    // 2. the strips: dequant + MFMA of the wave's chunks, partial tile to LDS,
    //    one barrier, the tile's reducer wave sums the WV partials in wave order
    // Every unrolled step issues its refill, past the last strip too (out of range:
    // no traffic): with a `break` the loop latch would also be reached right after
    // step 0's refill, and the waits at the loop head would drain the ring.
    // One reduction group (D = R strips, or D strips in R-sized groups) per call.
    // GU > 0 (two K slices, at most GU groups per workgroup): the groups are unrolled
    // so that each one's exchange results land in registers of their own (gotg[gi]),
    // and the reducer wave exchanges a group's sums as soon as they are summed: the
    // exchanges' traffic overlaps the next groups' dequant + MFMA instead of
    // following the last strip.
    uint64_t gotg[GU > 0 ? GU : 1][4];
#pragma unroll
    for (int gi = 0; gi < (GU > 0 ? GU : 1); ++gi)
#pragma unroll
        for (int q = 0; q < 4; ++q) gotg[gi][q] = 0;
    auto group = [&](uint32_t t0, uint64_t (&gg)[4]) __attribute__((always_inline)) {
        f32x4 accs[R][MT];  // the partials of the current reduction group (R strips)
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const uint32_t t = t0 + (uint32_t)d;
            const bool live = t < nst;  // uniform
            f32x4 (&acc)[MT] = accs[d % R];
            if (live) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
                if constexpr (KPW >= 2) {
#pragma unroll
                    for (int h = 0; h < KPW / 2; ++h) {
                        const u32x4 (&xs)[2][MT][4] = *reinterpret_cast<const u32x4 (*)[2][MT][4]>(&xf[2 * h]);
                        xr_pair_mma<DT, MT>(ring[d].w[2 * h], ring[d].w[2 * h + 1],
                                            qtab[ring[d].qa[h]] * ring[d].qb[h], ptab, slot8, xs, acc);
                    }
                }
                if (t == 0) NF4_GSTAMP(2);  // x and the first strip's weights arrived, first strip done
#pragma unroll
                for (int q = 0; q < (KPW >= 2 ? 0 : KPW); ++q) {
                    Chunk<MT, 1> ch;
                    ch.w[0] = ring[d].w[q];
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int s = 0; s < 4; ++s) ch.x[mt][s] = xf[q][mt][s];
                    const float scs[1] = {((float)ring[d].qa[q / 2] / 127.0f) * ring[d].qb[q / 2]};  // IEEE division (:45)
                    f32x4 a1[MT][1];
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) a1[mt][0] = acc[mt];
                    chunk_mma<DT, MT, 1>(ch, lut, scs, a1);
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) acc[mt] = a1[mt][0];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            xslot_issue<KPW>(A, s0 + t + (uint32_t)D, t + (uint32_t)D < nst, cw, ln, xm, ring[d]);
            __builtin_amdgcn_sched_barrier(0);
            if (d % R != R - 1) continue;  // the group's partials meet after its last strip
            const uint32_t tg = t + 1u - (uint32_t)R;  // first strip of the group
            if constexpr (!NF4_ABL_RED_ON) {
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) asm volatile("" ::"v"(accs[r][mt]));
            } else if (tg < nst) {  // uniform
                NF4_GSPAN_BEGIN();
                // red slot of strip u: ((u / R) & 1) * R + u % R (two groups in flight)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t u = tg + (uint32_t)r;
                    if (u < nst) {
                        f32x4* rb = red + (((u / R) & 1u) * R + (uint32_t)r) * (WV * MT * 64);
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt) rb[(wave * MT + mt) * 64 + lane] = accs[r][mt];
                    }
                }
                __syncthreads();
                NF4_GSPAN_END(7);  // partial tiles stored + the barrier
                NF4_GSPAN_BEGIN();
                if constexpr (GU > 0) {
                    // the one tile of the group this wave reduces (tile j = r MT + mt goes
                    // to wave (tg MT + j) mod WV, as below), with a single exchange site
                    // per result register: a merge of several sites made the compiler
                    // move the pending results between registers (a vmcnt(0) per move)
                    const uint32_t j = (wave + (uint32_t)WV - (tg * (uint32_t)MT) % (uint32_t)WV) % (uint32_t)WV;
                    const uint32_t r = j / (uint32_t)MT, mt = j % (uint32_t)MT, u = tg + r;
                    if (j < (uint32_t)(R * MT) && u < nst) {  // uniform
                        const f32x4* rb = red + (((u / R) & 1u) * R + r) * (WV * MT * 64);
                        f32x4 sum = rb[mt * 64 + lane];
#pragma unroll
                        for (int w = 1; w < WV; ++w) sum += rb[(w * MT + mt) * 64 + lane];
                        float* h = held + u * (16u * MT * 16u) + (16u * mt + 4u * kh) * 16u + nl;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            h[16u * q] = sum[q];
                            const float nb = __shfl_xor(sum[q], 1, 64);
                            const uint32_t m = 16u * mt + 4u * kh + q;
                            if (NF4_ABL_HANDOFF_ON && m < A.M && !(nl & 1u))
                                gg[q] = slab_swap2(A.slab + swap_entry(s0 + u, A.M, m, nl), sum[q], nb);
                        }
                    }
                    NF4_GSPAN_END(8);
                    continue;
                }
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t u = tg + (uint32_t)r;
                    const f32x4* rb = red + (((u / R) & 1u) * R + (uint32_t)r) * (WV * MT * 64);
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        if (u < nst && wave == (u * MT + (uint32_t)mt) % (uint32_t)WV) {  // uniform
                            f32x4 sum = rb[mt * 64 + lane];
#pragma unroll
                            for (int w = 1; w < WV; ++w) sum += rb[(w * MT + mt) * 64 + lane];
                            // sum[q] = Y[16 mt + 4 kh + q][strip col nl]
                            float* h = held + u * (16u * MT * 16u) + (16u * mt + 4u * kh) * 16u + nl;
#pragma unroll
                            for (int q = 0; q < 4; ++q) h[16u * q] = sum[q];
                        }
                    }
                }
                NF4_GSPAN_END(8);  // the reducer's sums
            }
        }
    };
    if constexpr (GU > 0) {
#pragma unroll
        for (int gi = 0; gi < GU; ++gi)
            if ((uint32_t)gi * (uint32_t)D < nst) group((uint32_t)gi * (uint32_t)D, gotg[gi]);  // uniform
    } else {
        for (uint32_t t0 = 0; t0 < nst; t0 += (uint32_t)D) group(t0, gotg[0]);
    }
    if constexpr (GU > 0 && !NF4_ABL_HANDOFF_ON) return;
    if constexpr (GU > 0) {
        // each reducer wave finishes its own tiles' exchanges: the second arriver sums
        // in slice order (its sums in `held`, written by this wave) and writes y
#pragma unroll
        for (int gi = 0; gi < GU; ++gi) {
            const uint32_t tg = (uint32_t)gi * (uint32_t)D;
            const uint32_t j = (wave + (uint32_t)WV - (tg * (uint32_t)MT) % (uint32_t)WV) % (uint32_t)WV;
            const uint32_t r = j / (uint32_t)MT, mt = j % (uint32_t)MT, u = tg + r;
            if (j >= (uint32_t)(R * MT) || u >= nst) continue;  // uniform: no tile of this wave
            {
                const uint32_t strip = s0 + u;
                const uint32_t mi = __builtin_amdgcn_readfirstlane(xr_mat_of(A, strip));
                uint16_t* const ybase = reinterpret_cast<uint16_t*>(A.mat[mi].y);
                const uint32_t yN = A.mat[mi].N, ycol = (strip - A.mat[mi].cg_begin) * 16u;
                {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint64_t g = gotg[gi][q];
                        if (g == 0) continue;  // not sent, or the first of the two
                        const uint32_t m = 16u * mt + 4u * kh + q;
                        const float* h = held + u * (16u * MT * 16u) + m * 16u + nl;
                        const float plo = __uint_as_float(~(uint32_t)g), phi = __uint_as_float(~(uint32_t)(g >> 32));
                        const float slo = ks == 0 ? h[0] + plo : plo + h[0];  // slice order
                        const float shi = ks == 0 ? h[1] + phi : phi + h[1];
                        *reinterpret_cast<uint32_t*>(ybase + m * yN + ycol + nl) = pack2<DT>(slo, shi);
                        __hip_atomic_store(A.slab + swap_entry(strip, A.M, m, nl), 0ull, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
        }
        return;
    }
    NF4_GSTAMP(3);
    __syncthreads();
    NF4_GSTAMP(4);

    // 3. the results: straight to y (one slice), or to the slab + tickets
    const uint32_t rows = A.M;
    if (S == 1) {
        // 16-bit pairs, a row's 16 columns = 8 consecutive dwords
        for (uint32_t e = tid; e < nst * rows * 8u; e += 64u * WV) {
            const uint32_t t = e / (rows * 8u), rem = e - t * rows * 8u, m = rem >> 3, p = rem & 7u;
            const uint32_t strip = s0 + t;
            const K128Mat& Mt = A.mat[xr_mat_of(A, strip)];
            const float* h = held + t * (16u * MT * 16u) + m * 16u + 2u * p;
            uint32_t* dst = reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(Mt.y) + m * Mt.N +
                                                        (strip - Mt.cg_begin) * 16u + 2u * p);
            *dst = pack2<DT>(h[0], h[1]);
        }
        NF4_GSTAMP(5);
        return;
    }
    if constexpr (!NF4_ABL_HANDOFF_ON) return;
    if (S == 2) {
        // two K slices (K <= 4096 at M > 16): hand-off by exchange (slab_swap2) in the
        // first slice's entries, kB swaps per thread in flight before any result is used
        constexpr int kB = 4;
        const uint32_t total = nst * rows * 8u;
        for (uint32_t e0 = tid; e0 < total; e0 += (uint32_t)kB * 64u * WV) {
            uint64_t got[kB];
            float lo[kB], hi[kB];
            uint32_t ent[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const uint32_t e = e0 + (uint32_t)b * 64u * WV;
                got[b] = 0;
                lo[b] = hi[b] = 0.0f;
                ent[b] = 0;
                if (e < total) {
                    const uint32_t t = e / (rows * 8u), rem = e - t * rows * 8u, m = rem >> 3, c = 2u * (rem & 7u);
                    const float* h = held + t * (16u * MT * 16u) + m * 16u + c;
                    lo[b] = h[0];
                    hi[b] = h[1];
                    ent[b] = swap_entry(s0 + t, A.M, m, c);
                    got[b] = slab_swap2(A.slab + ent[b], lo[b], hi[b]);
                }
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                if (got[b] == 0) continue;  // first of the two (or past the end): the partner finishes
                const uint32_t e = e0 + (uint32_t)b * 64u * WV;
                const uint32_t t = e / (rows * 8u), rem = e - t * rows * 8u, m = rem >> 3, p = rem & 7u;
                const float plo = __uint_as_float(~(uint32_t)got[b]), phi = __uint_as_float(~(uint32_t)(got[b] >> 32));
                const float slo = ks == 0 ? lo[b] + plo : plo + lo[b];  // slice order
                const float shi = ks == 0 ? hi[b] + phi : phi + hi[b];
                const uint32_t strip = s0 + t;
                const K128Mat& Mt = A.mat[xr_mat_of(A, strip)];
                uint32_t* dst = reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(Mt.y) + m * Mt.N +
                                                            (strip - Mt.cg_begin) * 16u + 2u * p);
                *dst = pack2<DT>(slo, shi);
                __hip_atomic_store(A.slab + ent[b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        NF4_GSTAMP(5);
        NF4_GSTAMP(9);
        return;
    }
    // slab [ks][M][ncols] entries (strip s at columns 16 s): splitk_ticket / splitk_reduce
    for (uint32_t e = tid; e < nst * rows * 8u; e += 64u * WV) {  // column pairs
        const uint32_t t = e / (rows * 8u), rem = e - t * rows * 8u, m = rem >> 3, c = 2u * (rem & 7u);
        const float* h = held + t * (16u * MT * 16u) + m * 16u + c;
        slab_put2(A.slab, slab_entry(ks, A.M, m, A.ncols, (s0 + t) * 16u + c), h[0], h[1]);
    }
    // no wait for the entries' write acknowledgements before the tickets: the
    // reducer polls every entry until it is written, so a ticket only says who sums
    // (waiting cost a memory round trip per launch)
    NF4_GSTAMP(5);
    __syncthreads();
    if (tid < nst) last_flags[tid] = splitk_ticket(&A.counters[s0 + tid], S);  // one ticket per strip; nst <= 64
    __syncthreads();
    for (uint32_t t = wave; t < nst; t += (uint32_t)WV) {
        if (!last_flags[t]) continue;  // uniform
        const uint32_t strip = s0 + t;
        const K128Mat& Mt = A.mat[xr_mat_of(A, strip)];
        const uint32_t lc = (strip - Mt.cg_begin) * 16u;
        NF4_GSTAMP(6);  // tickets drawn: this wave reduces (the last arriver)
        splitk_reduce<DT, 16u>(A.slab, S, A.M, A.ncols, strip * 16u, Mt.y, Mt.N, lc, lane, A.counters);
    }
    NF4_GSTAMP(9);
}

template <int DT, int MT, int WV, int KPW, int D, int GU>
__global__ __launch_bounds__(64 * WV) void nf4_gemm_xr_kernel(const GemmArgs A) {
    xr_body<DT, MT, WV, KPW, D, GU>(A);
}
// GU > 0: the unrolled groups keep 4 x 4 exchange results per lane live across the
// loop; at one workgroup of 8 waves per CU (2 per SIMD) the kernel may use up to
// 256 registers, and with the default budget the allocator moved those results
// between registers (each move a full vmcnt(0) drain inside the ring)
template <int DT, int MT, int WV, int KPW, int D, int GU>
__global__ __launch_bounds__(64 * WV) __attribute__((amdgpu_waves_per_eu(1, 2))) void nf4_gemm_xrg_kernel(
    const GemmArgs A) {
    xr_body<DT, MT, WV, KPW, D, GU>(A);
}

// ---------------------------------------------------------------------------
// Streaming decode kernel (K % 256 == 0).  Weight bytes are the only operand
// that comes from HBM, so a wave keeps P chunks of them in flight in registers
// (a ring refilled right after each chunk is consumed: counted vmcnt, never a
// drain) and takes everything else from LDS: the activation slice x[0:M, k0:k1]
// is staged once per workgroup, the 16 NF4 codes and the 256 values q/127 are
// tables there.  A chunk is 256 deep: one 128-byte line of each of the strip's
// 16 weight rows; lane (nl, kh) holds 32 bytes = exactly one 64-block (one
// scale) of row nl, i.e. eight MFMA B fragments.  Waves of a workgroup split
// the strip's K slice (interleaved chunks, so neighbouring waves read
// neighbouring lines) and T strips; partial sums meet in LDS in a fixed order.
constexpr uint32_t kSChunkK = 256;

constexpr int kXR = 8;               // x staging: 16-byte pieces per thread and row tile
constexpr uint32_t kLdsX = 0;        // dynamic LDS: [x slice][zero block][partials]

// One weight of a launch.  Several weights that share x (q/k/v, gate/up) go in
// one launch: workgroups are numbered over all their strip groups.
constexpr int kGroupMax = 8;
struct StreamMat {
    const uint8_t* packed;
    const uint8_t* a1;
    const float* a2;
    void* y;                // [M][N]
    uint32_t N;
    uint32_t sg_begin;      // first strip group of this weight in the launch
    uint32_t strip_begin;   // first 16-column strip (ticket counters), = col_begin / 16
    uint32_t nb_bytes, n2_bytes;
    FastDiv nb, n2;
};

struct StreamArgs {
    StreamMat mat[kGroupMax];
    uint32_t nmat;
    uint32_t sg_total;      // strip groups over all weights
    uint32_t ncols;         // sum of N (split-K slab row length)
    const void* x;
    uint64_t* slab;
    uint32_t* counters;
    uint32_t M, K;
    uint32_t T, parts;      // strips per workgroup, K parts per strip
    uint32_t ksplit, cps;   // K slices, chunks per slice
    uint32_t cpp;           // chunks per K part (a part's chunks are contiguous)
    uint32_t chunks;        // K / 256
    uint32_t bpr, groups;   // K / 64, ceil(bpr / 4)
    FastDiv ppr;            // 16-byte x pieces per staged row (cps * 32)
    uint32_t xstride;       // LDS bytes per staged x row
    uint32_t zero_off;      // 128 zero bytes: the A operand of rows >= M
    uint32_t red_off;       // [W][MT][64] f32x4 partial sums (persistent: two sets)
    uint32_t out_off;       // persistent: finished outputs [group][strip][M][16] (16-bit)
};

struct SSlot {
    u32x4 w0, w1;
    uint32_t qa;
    float qb;
};

constexpr int kVsMax = 16;  // chunks per wave covered by the vector-scale form  // beyond every buffer range: loads return 0, no traffic

template <bool VS>
__device__ __forceinline__ void sslot_issue(const StreamArgs& A, const StreamMat& Mt, __amdgpu_buffer_rsrc_t rw,
                                            __amdgpu_buffer_rsrc_t ra1, __amdgpu_buffer_rsrc_t ra2, uint32_t c,
                                            bool valid, uint32_t row, uint32_t kh, SSlot& s) {
    // `valid` is wave-uniform; past the wave's last chunk the offsets get bit 31
    // (beyond every range: zeros, no traffic) -- arithmetic, not a branch, so
    // the waitcnt pass sees one straight-line ring
    const uint32_t oob = valid ? 0u : kOob;
    const uint32_t woff = (row * (A.K >> 1) + c * 128u + kh * 32u) | oob;
    s.w0 = NF4_ABL_WLOAD(rw, woff);
    s.w1 = NF4_ABL_WLOAD(rw, woff + 16u);
    if constexpr (!VS) {
        // block 4c + kh of the row; its nested group is c (reference wraps, :173-186)
        const uint32_t i1 = fmodu(row * A.bpr + 4u * c + kh, Mt.nb) | oob;
        const uint32_t i2 = (fmodu(row * A.groups + c, Mt.n2) * 4u) | oob;
        s.qa = __builtin_amdgcn_raw_buffer_load_b8(ra1, i1, 0, 0);
        s.qb = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra2, i2, 0, 0));
    }
}

// The dequant body: codes are looked up in pairs from a 256-entry table
// (code[b >> 4], code[b & 15]) per packed byte b, replicated into 32 lane slots
// so that lane l reads bank pair 2 (l mod 32): one conflict-free ds_read_b64
// per two weights, its LDS address one v_perm_b32 (byte b into bits 8..15, the
// lane's slot offset into bits 0..7).  Then the fp32 products with the block
// scale and one RNE pack per pair: 1.5 VALU per weight.
template <int DT, int MT, bool SC = false>  // SC: qb is the block scale itself (qtab unused)
__device__ __forceinline__ void sslot_mma(const SSlot& s, uint32_t qa, float qb, const f32x2* ptab,
                                          const float* qtab, const char* smem, uint32_t slot8,
                                          const uint32_t (&xa)[MT], f32x4 (&acc)[MT], f32x4 (&accb)[MT]) {
    // even steps accumulate into acc, odd into accb: two MFMA dependency chains of 4
    const float sc = SC ? qb : qtab[qa] * qb;  // (:45, :97-98)
    // both halves materialised: a half left to op_sel would read a stale
    // register, and its pending load (as far as the waitcnt pass knows) drains the ring
    const f32x2 sc2 = {sc, opaque(sc)};
    const char* pt = reinterpret_cast<const char*>(ptab);
    // Pair lookups run LA steps ahead of their use (one LDS round trip per chunk,
    // not one per MFMA step): 4 x LA reads in flight, counted lgkmcnt waits.
    constexpr int LA = 3;
    f32x2 v[8][4];
    auto issue = [&](int st) {
        const uint32_t wd = st < 4 ? s.w0[st] : s.w1[st - 4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t addr = __builtin_amdgcn_perm(wd, slot8, 0x0C0C0000u | ((4u + b) << 8));
            v[st][b] = NF4_ABL_LOOKUP(pt, addr, wd);
        }
    };
#pragma unroll
    for (int st = 0; st < LA; ++st) issue(st);
#pragma unroll
    for (int st = 0; st < 8; ++st) {
        if (st + LA < 8) issue(st + LA);
        u32x4 a[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a[mt] = NF4_ABL_XFRAG(smem, xa[mt] + 16u * st);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t bw[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const f32x2 p = v[st][b] * sc2;  // fp32 products (:97-98)
            bw[b] = pack2<DT>(p.x, p.y);     // RNE (:109-110)
        }
        const u32x4 bq = {bw[0], bw[1], bw[2], bw[3]};
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            f32x4& c = (st & 1) ? accb[mt] : acc[mt];
            if constexpr (!NF4_ABL_MMA_ON) {
                asm volatile("" ::"v"(a[mt]), "v"(bq));
            } else if constexpr (DT == NF4DQ_BF16) {
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[mt]),
                                                            __builtin_bit_cast(bf16x8, bq), c, 0, 0, 0);
            } else {
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a[mt]),
                                                           __builtin_bit_cast(f16x8, bq), c, 0, 0, 0);
            }
        }
    }
}

// Two chunks of one strip (one row tile, M <= 16) decoded step by step side by
// side: two independent chains of pair lookups, x reads and MFMAs, so that one
// chunk's LDS round trips overlap the other's VALU work.  Scales come in computed.
template <int DT>
__device__ __forceinline__ void sslot_mma_pair(const SSlot& s0, const SSlot& s1, float scA, float scB,
                                               const f32x2* ptab, const char* smem, uint32_t slot8, uint32_t xaA,
                                               uint32_t xaB, f32x4& acc, f32x4& accb) {
    const f32x2 sA = {scA, opaque(scA)}, sB = {scB, opaque(scB)};
    const char* pt = reinterpret_cast<const char*>(ptab);
    constexpr int LA = 2;
    f32x2 vA[8][4], vB[8][4];
    auto issue = [&](int st) {
        const uint32_t wa = st < 4 ? s0.w0[st] : s0.w1[st - 4];
        const uint32_t wb = st < 4 ? s1.w0[st] : s1.w1[st - 4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t sel = 0x0C0C0000u | ((4u + b) << 8);
            vA[st][b] = NF4_ABL_LOOKUP(pt, __builtin_amdgcn_perm(wa, slot8, sel), wa);
            vB[st][b] = NF4_ABL_LOOKUP(pt, __builtin_amdgcn_perm(wb, slot8, sel), wb);
        }
    };
#pragma unroll
    for (int st = 0; st < LA; ++st) issue(st);
#pragma unroll
    for (int st = 0; st < 8; ++st) {
        if (st + LA < 8) issue(st + LA);
        const u32x4 a0 = *reinterpret_cast<const u32x4*>(smem + xaA + 16u * st);
        const u32x4 a1 = *reinterpret_cast<const u32x4*>(smem + xaB + 16u * st);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t bw0[4], bw1[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const f32x2 p0 = vA[st][b] * sA, p1 = vB[st][b] * sB;  // fp32 products (:97-98)
            bw0[b] = pack2<DT>(p0.x, p0.y);                          // RNE (:109-110)
            bw1[b] = pack2<DT>(p1.x, p1.y);
        }
        const u32x4 bq0 = {bw0[0], bw0[1], bw0[2], bw0[3]}, bq1 = {bw1[0], bw1[1], bw1[2], bw1[3]};
        if constexpr (!NF4_ABL_MMA_ON) {
            asm volatile("" ::"v"(a0), "v"(a1), "v"(bq0), "v"(bq1));
        } else if constexpr (DT == NF4DQ_BF16) {
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a0), __builtin_bit_cast(bf16x8, bq0),
                                                          acc, 0, 0, 0);
            accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a1),
                                                           __builtin_bit_cast(bf16x8, bq1), accb, 0, 0, 0);
        } else {
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a0), __builtin_bit_cast(f16x8, bq0),
                                                         acc, 0, 0, 0);
            accb = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a1), __builtin_bit_cast(f16x8, bq1),
                                                          accb, 0, 0, 0);
        }
    }
}

// VS: vector scales -- no absmax wrap inside a row (nb a multiple of K / 64 or
// >= N K / 64, n2 a multiple of groups or >= N groups: true for every real
// bitsandbytes state, where n2 = N groups / 64) and at most kVsMax chunks per wave: the wave's absmax bytes (4 per chunk) and nested
// scales (1 per chunk) come in 16-byte loads up front instead of two gathers
// per chunk, and the chunk loop is unrolled so that every index is static.
template <int DT, int MT, int W, int P, bool VS>
__global__ __launch_bounds__(64 * W) void nf4_gemm_stream_kernel(const StreamArgs A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ __attribute__((aligned(16))) f32x2 ptab[256 * 32];  // 64 KiB pair table, built per workgroup
    __shared__ float qtab[256];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar control flow below
    const uint32_t nl = lane & 15u, kh = lane >> 4;
    const uint32_t sgi = blockIdx.x % A.sg_total, ks = blockIdx.x / A.sg_total;
    uint32_t mi = 0;  // the weight this workgroup works on (uniform scan)
    for (uint32_t i = 1; i < A.nmat; ++i) mi = sgi >= A.mat[i].sg_begin ? i : mi;
    const StreamMat& Mt = A.mat[mi];
    const uint32_t sg = sgi - Mt.sg_begin;
    const uint32_t strip = sg * A.T + wave % A.T, part = wave / A.T;
    const uint32_t row = strip * 16u + nl;
    // an empty last slice (ksplit * cps > chunks, e.g. 5 chunks in 4 slices of 2): s0 is
    // clamped, so the slice has no chunks, contributes zero partials and takes its ticket
    const uint32_t s0r = ks * A.cps, s0 = s0r < A.chunks ? s0r : A.chunks;
    const uint32_t s1 = s0 + A.cps < A.chunks ? s0 + A.cps : A.chunks;
    const uint32_t nloc = s1 - s0;
    const uint32_t l0 = part * A.cpp;  // first chunk of this wave within the slice
    const uint32_t cnt = nloc > l0 ? (nloc - l0 < A.cpp ? nloc - l0 : A.cpp) : 0u;
    NF4_GSTAMP_INIT(W);
    NF4_GSTAMP(0);

    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.packed, 0, Mt.N * (A.K >> 1), kRsrcFlags);
    const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.a1, 0, Mt.nb_bytes, kRsrcFlags);
    const __amdgpu_buffer_rsrc_t ra2 = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.a2, 0, Mt.n2_bytes, kRsrcFlags);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, 0, A.M * A.K * 2u, kRsrcFlags);

    // 1. activation slice loads first (the counted waits below then leave the weight ring in flight)
    const uint32_t pieces = A.M * A.ppr.d;
    constexpr int XR = kXR * MT;
    u32x4 xv[XR];
    uint32_t xdst[XR];
#pragma unroll
    for (int i = 0; i < XR; ++i) {
        const uint32_t p = tid + (uint32_t)i * 64u * W;
        const uint32_t r = fdiv(p, A.ppr), q = p - r * A.ppr.d;
        const bool ok = p < pieces && s0 * 256u + q * 8u < A.K;
        xv[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? (r * A.K + s0 * 256u) * 2u + q * 16u : kOob, 0, 0);
        xdst[i] = p < pieces ? kLdsX + r * A.xstride + q * 16u : 0xFFFFFFFFu;
    }
    // 2. the weight ring (VS: the wave's scales first)
    // (issue order = the loop's: slot by slot, w0 w1 qa qb -- the scheduler must
    // not regroup them, or the waitcnt pass merges two orders into a drain)
    // VS: scales of 4 chunks per 16-byte pair of loads, two groups live (the
    // next group's pair is issued as the current one starts)
    u32x4 a1v[2], a2v[2];
    uint32_t b1 = 0, b2 = 0;
    auto scale_issue = [&](int g) {
        const uint32_t oob = 4u * g < cnt ? 0u : kOob;  // groups past the wave's range: no traffic
        a1v[g & 1] = __builtin_amdgcn_raw_buffer_load_b128(ra1, (b1 + 16u * g) | oob, 0, 0);
        a2v[g & 1] = __builtin_amdgcn_raw_buffer_load_b128(ra2, ((b2 + 4u * g) * 4u) | oob, 0, 0);
    };
    if constexpr (VS) {
        const uint32_t cf = s0 + l0;
        // the row's wrapped bases (reference repeat semantics, :173-186); no wrap inside the row
        b1 = fmodu(row * A.bpr, Mt.nb) + 4u * cf;
        b2 = fmodu(row * A.groups, Mt.n2) + cf;
        scale_issue(0);
        __builtin_amdgcn_sched_barrier(0);
    }
    SSlot ring[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        sslot_issue<VS>(A, Mt, rw, ra1, ra2, s0 + l0 + (uint32_t)j, (uint32_t)j < cnt, row, kh, ring[j]);
        __builtin_amdgcn_sched_barrier(0);
    }
    // 3. tables (no global data: they fill while the loads fly), then the staged
    // slice (waits for the x loads only), one barrier.  Pair table: entry
    // e = 16 hi + lo of lane slot t at byte 256 e + 8 t; a thread owns one
    // (lo, t) and writes it for all 16 hi -- the hi codes are immediates.
    if (tid < 256u) qtab[tid] = (float)tid / 127.0f;  // IEEE division
    if (tid < 8u) *reinterpret_cast<u32x4*>(smem + A.zero_off + 16u * tid) = u32x4{0u, 0u, 0u, 0u};
    for (uint32_t u = tid; u < 16u * 32u; u += 64u * W) {
        const float clo = nf4_code(u >> 5);
#pragma unroll
        for (int hi = 0; hi < 16; ++hi) ptab[(16u * hi + (u >> 5)) * 32u + (u & 31u)] = f32x2{nf4_code(hi), clo};
    }
#pragma unroll
    for (int i = 0; i < XR; ++i)
        if (xdst[i] != 0xFFFFFFFFu) *reinterpret_cast<u32x4*>(smem + xdst[i]) = xv[i];
    __syncthreads();
    NF4_GSTAMP(1);

    uint32_t xa0[MT];
    bool live[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        live[mt] = 16u * mt + nl < A.M;
        xa0[mt] = live[mt] ? kLdsX + (16u * mt + nl) * A.xstride + kh * 128u : A.zero_off;
    }
    const uint32_t slot8 = (lane & 31u) * 8u;
    f32x4 acc[MT], accb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = accb[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto body = [&](uint32_t jj, int j, uint32_t qa, float qb) {
        const uint32_t l = l0 + jj;  // chunk within the slice
        uint32_t xa[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xa[mt] = live[mt] ? xa0[mt] + l * 512u : xa0[mt];
        sslot_mma<DT, MT>(ring[j], qa, qb, ptab, qtab, smem, slot8, xa, acc, accb);
    };
    if constexpr (VS) {
        // fully unrolled: ring slot jj % P, scale lanes jj / 4 and jj % 4 are static
#pragma unroll
        for (int jj = 0; jj < kVsMax; ++jj) {
            const int j = jj % P;
            if (jj % 4 == 0 && jj + 4 < kVsMax) {
                scale_issue(jj / 4 + 1);
                __builtin_amdgcn_sched_barrier(0);
            }
            if ((uint32_t)jj < cnt)  // uniform
                body((uint32_t)jj, j, (a1v[(jj / 4) & 1][jj % 4] >> (8u * kh)) & 0xFFu,
                     __uint_as_float(a2v[(jj / 4) & 1][jj % 4]));
            __builtin_amdgcn_sched_barrier(0);
            // unconditional (past the range: out-of-range offsets, no traffic), so
            // both sides of the guard leave the same loads pending
            const uint32_t jn = (uint32_t)jj + P;
            sslot_issue<VS>(A, Mt, rw, ra1, ra2, s0 + l0 + jn, jn < cnt, row, kh, ring[j]);
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
        for (uint32_t base = 0; base < cnt; base += P) {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const uint32_t jj = base + (uint32_t)j;
                if (jj < cnt) body(jj, j, ring[j].qa, ring[j].qb);
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t jn = jj + P;
                sslot_issue<VS>(A, Mt, rw, ra1, ra2, s0 + l0 + jn, jn < cnt, row, kh, ring[j]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }

#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] += accb[mt];
    NF4_GSTAMP(2);
    // 4. the strip's K parts meet in LDS, in part order (the partials reuse the
    // x slice's LDS once every wave is done reading it)
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(smem + A.red_off);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[(wave * MT + mt) * 64u + lane] = acc[mt];
    __syncthreads();
    if (part != 0) return;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        f32x4 s = red[(wave * MT + mt) * 64u + lane];
        for (uint32_t p = 1; p < A.parts; ++p) s += red[((wave + p * A.T) * MT + mt) * 64u + lane];
        acc[mt] = s;
    }
    // acc[mt][r] = Y[16 mt + 4 kh + r][row]
    if (A.ksplit == 1) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t m = 16u * mt + 4u * kh + r;
                if (m < A.M) store_y<DT>(Mt.y, m * Mt.N + row, acc[mt][r]);
            }
        NF4_GSTAMP(3);
        return;
    }
    // 5. split-K across workgroups: the hand-off of nf4_gemm_smallm_kernel, per strip
    const uint32_t gstrip = Mt.strip_begin + strip;  // launch-wide strip: counter and slab column
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t m = 16u * mt + 4u * kh + r;
            slab_put_lane(A.slab, slab_entry(ks, A.M, m, A.ncols, gstrip * 16u + nl), acc[mt][r], nl, m < A.M);
        }
    uint32_t last = 0;
    if (lane == 0) last = splitk_ticket(&A.counters[gstrip], A.ksplit);
    last = __builtin_amdgcn_readfirstlane(last);
    if (!last) return;
    splitk_reduce<DT, 16u>(A.slab, A.ksplit, A.M, A.ncols, gstrip * 16u, Mt.y, Mt.N, strip * 16u, lane, A.counters);
}


// ---------------------------------------------------------------------------
// Persistent form of the streaming kernel (M <= 16, whole-K activation rows in
// LDS, absmax without in-row wrap).  One workgroup per CU walks strip groups
// (of every weight of a grouped launch) with a grid stride; each wave's ring
// runs on ACROSS groups, so a launch pays the first-data latency, the LDS
// tables and the activation staging once per CU instead of once per
// workgroup.  The ring advances a round (P chunks) at a time; the absmax bytes
// and nested scales of a round come in two loads issued ahead of its weights.
// Finished groups are combined in LDS (double-buffered, one barrier per group)
// and held there until the end, so that no global store sits between the
// ring's loads (a store would turn every counted wait into a drain).
template <int P>
struct PScales {
    typedef uint32_t vec __attribute__((ext_vector_type(P)));
    vec a1, a2;
};

template <int P>
__device__ __forceinline__ typename PScales<P>::vec pload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    if constexpr (NF4_ABL_PLOAD_FAKE) {  // tools: scales made from the offset (no gather)
        typename PScales<P>::vec v;
#pragma unroll
        for (int i = 0; i < P; ++i) v[i] = 0x3C000000u | ((off * 37u + (uint32_t)i) & 0x7F7Fu);
        return v;
    } else if constexpr (P == 2) return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    else return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

struct PGeo {  // where the ring issues: one strip of one weight
    __amdgpu_buffer_rsrc_t rw, ra1, ra2;
    uint32_t row, b1, b2;
    uint32_t wbase;  // the lane's first weight byte of the slice: row K / 2 + kh 32 + chunk base 128
};

template <int DT, int W, int P, bool SPLIT>
__global__ __launch_bounds__(64 * W) void nf4_gemm_persist_kernel(const StreamArgs A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ __attribute__((aligned(16))) f32x2 ptab[256 * 32];
    __shared__ float qtab[256];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t nl = lane & 15u, kh = lane >> 4;
    const uint32_t strip_in = wave % A.T, part = wave / A.T;
    if constexpr (NF4_ABL_ENTRY_RETURN) return;
    // K slices: workgroup b works on slice b % ksplit (its x slice staged once),
    // walking the strip groups b / ksplit, + G / ksplit, ...
    const uint32_t KS = SPLIT ? A.ksplit : 1u, ks = SPLIT ? blockIdx.x % KS : 0u;
    const uint32_t G = gridDim.x / KS, j0 = blockIdx.x / KS;
    const uint32_t mine = A.sg_total > j0 ? (A.sg_total - j0 + G - 1u) / G : 0u;
    const uint32_t cnt = A.cpp;  // chunks per wave per group (host: parts * cnt == cps, cnt % P == 0)
    const uint32_t rounds = cnt / P, total = mine * rounds;
    const uint32_t l0 = part * cnt;          // first chunk of this wave within the slice
    const uint32_t cbase = ks * A.cps;       // first chunk of the slice within K
    NF4_GSTAMP_INIT(W);
    NF4_GSTAMP(0);

    auto geo = [&](uint32_t it, PGeo& g) {
        const uint32_t sgi = j0 + it * G;
        uint32_t mi = 0;
        for (uint32_t i = 1; i < A.nmat; ++i) mi = sgi >= A.mat[i].sg_begin ? i : mi;
        const StreamMat& Mt = A.mat[mi];
        g.row = ((sgi - Mt.sg_begin) * A.T + strip_in) * 16u + nl;
        g.rw = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.packed, 0, Mt.N * (A.K >> 1), kRsrcFlags);
        g.ra1 = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.a1, 0, Mt.nb_bytes, kRsrcFlags);
        g.ra2 = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.a2, 0, Mt.n2_bytes, kRsrcFlags);
        g.b1 = fmodu(g.row * A.bpr, Mt.nb) + 4u * (cbase + l0);  // reference wrap (:173-186), none inside a row
        g.b2 = fmodu(g.row * A.groups, Mt.n2) + cbase + l0;
        g.wbase = g.row * (A.K >> 1) + (cbase + l0) * 128u + kh * 32u;
    };
    // issue pointer: group it2, round rr2 of it
    PGeo gi;
    uint32_t it2 = 0, rr2 = 0;
    geo(0, gi);
    auto issue_scales = [&](PScales<P>& sc, bool valid) {
        const uint32_t oob = valid ? 0u : kOob;
        sc.a1 = pload<P>(gi.ra1, (gi.b1 + 4u * P * rr2) | oob);
        sc.a2 = pload<P>(gi.ra2, ((gi.b2 + P * rr2) * 4u) | oob);
    };
    auto issue_w = [&](SSlot& sl, int s, bool valid) {
        const uint32_t woff = (gi.wbase + (rr2 * P + (uint32_t)s) * 128u) | (valid ? 0u : kOob);
        sl.w0 = NF4_ABL_WLOAD(gi.rw, woff);
        sl.w1 = NF4_ABL_WLOAD(gi.rw, woff + 16u);
    };
    auto advance = [&]() {  // uniform
        if (++rr2 == rounds) {
            rr2 = 0;
            ++it2;
            if (it2 < mine) geo(it2, gi);
        }
    };

    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, 0, A.M * A.K * 2u, kRsrcFlags);
    // 1. x rows (the slice's K range), then round 0 of the ring
    const uint32_t pieces = A.M * A.ppr.d;
    u32x4 xv[kXR];
    uint32_t xdst[kXR];
#pragma unroll
    for (int i = 0; i < kXR; ++i) {
        const uint32_t p = tid + (uint32_t)i * 64u * W;
        const uint32_t r = fdiv(p, A.ppr), q = p - r * A.ppr.d;
        xv[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, p < pieces ? r * A.K * 2u + cbase * 512u + q * 16u : kOob,
                                                      0, 0);
        xdst[i] = p < pieces ? kLdsX + r * A.xstride + q * 16u : 0xFFFFFFFFu;
    }
    __builtin_amdgcn_sched_barrier(0);  // x loads first: the staging below must not wait on the ring
    PScales<P> sc[2];
    SSlot ring[P];
    issue_scales(sc[0], total > 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < P; ++s) {
        issue_w(ring[s], s, total > 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    advance();
    // 2. tables while the loads fly, then the x rows, one barrier
    if (tid < 256u) qtab[tid] = (float)tid / 127.0f;
    if (tid < 8u) *reinterpret_cast<u32x4*>(smem + A.zero_off + 16u * tid) = u32x4{0u, 0u, 0u, 0u};
    for (uint32_t u = tid; u < 16u * 32u; u += 64u * W) {
        const float clo = nf4_code(u >> 5);
#pragma unroll
        for (int hi = 0; hi < 16; ++hi) ptab[(16u * hi + (u >> 5)) * 32u + (u & 31u)] = f32x2{nf4_code(hi), clo};
    }
#pragma unroll
    for (int i = 0; i < kXR; ++i)
        if (xdst[i] != 0xFFFFFFFFu) *reinterpret_cast<u32x4*>(smem + xdst[i]) = xv[i];
    __syncthreads();
    NF4_GSTAMP(1);

    const bool live = nl < A.M;
    const uint32_t xa0 = live ? kLdsX + nl * A.xstride + kh * 128u : A.zero_off;
    const uint32_t slot8 = (lane & 31u) * 8u;
    f32x4 acc[1] = {f32x4{0.f, 0.f, 0.f, 0.f}}, accb[1] = {f32x4{0.f, 0.f, 0.f, 0.f}};
    uint32_t it = 0, rr = 0, buf = 0;

    auto round = [&](PScales<P>& cur, PScales<P>& nxt) {
        const bool more = it2 < mine;  // the issue pointer is one round ahead
        issue_scales(nxt, more);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (NF4_PERSIST_PAIR && P % 2 == 0) {
#pragma unroll
            for (int s = 0; s < P; s += 2) {
                const uint32_t l = l0 + rr * P + (uint32_t)s;
                const uint32_t xa = live ? xa0 + l * 512u : xa0, xb = live ? xa + 512u : xa0;
                const float scA = qtab[(cur.a1[s] >> (8u * kh)) & 0xFFu] * __uint_as_float(cur.a2[s]);  // (:45, :97-98)
                const float scB = qtab[(cur.a1[s + 1] >> (8u * kh)) & 0xFFu] * __uint_as_float(cur.a2[s + 1]);
                sslot_mma_pair<DT>(ring[s], ring[s + 1], scA, scB, ptab, smem, slot8, xa, xb, acc[0], accb[0]);
                if (it == 0 && rr == 0 && s == 0) NF4_GSTAMP(2);
                __builtin_amdgcn_sched_barrier(0);
                issue_w(ring[s], s, more);
                __builtin_amdgcn_sched_barrier(0);
                issue_w(ring[s + 1], s + 1, more);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
            // the round's block scales in one LDS round trip, ahead of its first chunk
            // (not one dependent qtab read per chunk: 0.6-2 % per launch, round 4)
            float scv[P];
#pragma unroll
            for (int s = 0; s < P; ++s)
                scv[s] = qtab[(cur.a1[s] >> (8u * kh)) & 0xFFu] * __uint_as_float(cur.a2[s]);  // (:45, :97-98)
#pragma unroll
            for (int s = 0; s < P; ++s) {
                const uint32_t l = l0 + rr * P + (uint32_t)s;
                const uint32_t xa[1] = {live ? xa0 + l * 512u : xa0};
                sslot_mma<DT, 1, true>(ring[s], 0u, scv[s], ptab, qtab, smem, slot8, xa, acc, accb);
                if (it == 0 && rr == 0 && s == 0) NF4_GSTAMP(2);  // first chunk's weights arrived and consumed
                __builtin_amdgcn_sched_barrier(0);
                issue_w(ring[s], s, more);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        advance();
        if (++rr == rounds) {  // group `it` done (uniform)
            f32x4* red = reinterpret_cast<f32x4*>(smem + A.red_off) + buf * (64u * W);
            NF4_GSPAN_BEGIN();
            red[wave * 64u + lane] = acc[0] + accb[0];
            __syncthreads();
            NF4_GSPAN_END(7);
            if (part == 0) {
                f32x4 sum = red[wave * 64u + lane];
                for (uint32_t q = 1; q < A.parts; ++q) sum += red[(wave + q * A.T) * 64u + lane];
                const uint32_t o0 = ((it * A.T + strip_in) * A.M) * 16u;
                if constexpr (!SPLIT) {  // finished: the 16-bit outputs
                    uint16_t* o = reinterpret_cast<uint16_t*>(smem + A.out_off) + o0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t m = 4u * kh + r;
                        if (m < A.M) o[m * 16u + nl] = (uint16_t)(pack2<DT>(sum[r], 0.0f) & 0xFFFFu);
                    }
                } else {  // this slice's fp32 partial sums
                    float* o = reinterpret_cast<float*>(smem + A.out_off) + o0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t m = 4u * kh + r;
                        if (m < A.M) o[m * 16u + nl] = sum[r];
                    }
                }
            }
            acc[0] = accb[0] = f32x4{0.f, 0.f, 0.f, 0.f};
            buf ^= 1u;
            rr = 0;
            ++it;
        }
    };
    for (uint32_t g = 0; g < (NF4_ABL_LOOP_ON ? total : 0u); g += 2) {
        round(sc[0], sc[1]);
        if (g + 1 < total) round(sc[1], sc[0]);
    }
    // 3. the workgroup's outputs
    NF4_GSTAMP(3);
    __syncthreads();
    NF4_GSTAMP(4);
    const uint32_t per = A.T * A.M * 16u;
    if constexpr (!SPLIT) {
        // one held strip per wave at a time: wave w stores strips w, w + W, ... of the
        // workgroup's (group, strip) list, [M][16] values 64 per pass (T is 1, 2 or 4:
        // no divisions; the weight is a uniform scan)
        const uint16_t* o = reinterpret_cast<const uint16_t*>(smem + A.out_off);
        const uint32_t tsh = A.T == 4u ? 2u : A.T == 2u ? 1u : 0u;
        for (uint32_t q = wave; q < (mine << tsh); q += W) {
            const uint32_t ito = q >> tsh, t = q & (A.T - 1u);
            const uint32_t sgi = j0 + ito * G;
            uint32_t mi = 0;
            for (uint32_t j = 1; j < A.nmat; ++j) mi = sgi >= A.mat[j].sg_begin ? j : mi;
            const StreamMat& Mt = A.mat[mi];
            const uint32_t col0 = ((sgi - Mt.sg_begin) * A.T + t) * 16u;
            const uint16_t* os = o + q * A.M * 16u;  // (ito T + t) M 16
            for (uint32_t e = lane; e < A.M * 16u; e += 64u)
                reinterpret_cast<uint16_t*>(Mt.y)[(e >> 4) * Mt.N + col0 + (e & 15u)] = os[e];
        }
        NF4_GSTAMP(5);
    } else {
    // 3b. K slices: the partials to the slab [ksplit][M][ncols], then per strip
    // group a ticket; the slice drawing ksplit - 1 sums all slices in slice order
    // (splitk_ticket / splitk_reduce)
    const float* o32 = reinterpret_cast<const float*>(smem + A.out_off);
    if (KS == 2) {
        // two slices: hand-off by exchange (slab_swap2) in the first slice's entries,
        // kB swaps per thread in flight before any result is used
        constexpr int kB = 4;
        for (uint32_t i0 = 2u * tid; i0 < mine * per; i0 += (uint32_t)kB * 2u * 64u * W) {
            uint64_t got[kB];
            uint32_t ent[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const uint32_t i = i0 + (uint32_t)b * 2u * 64u * W;
                got[b] = 0;
                ent[b] = 0;
                if (i < mine * per) {
                    const uint32_t ito = i / per, rem = i - ito * per;
                    const uint32_t t = rem / (A.M * 16u), rem2 = rem - t * (A.M * 16u);
                    const uint32_t sgi = j0 + ito * G;
                    uint32_t mi = 0;
                    for (uint32_t j = 1; j < A.nmat; ++j) mi = sgi >= A.mat[j].sg_begin ? j : mi;
                    const uint32_t gstrip = A.mat[mi].strip_begin + (sgi - A.mat[mi].sg_begin) * A.T + t;
                    ent[b] = swap_entry(gstrip, A.M, rem2 >> 4, rem2 & 15u);
                    got[b] = slab_swap2(A.slab + ent[b], o32[i], o32[i + 1]);
                }
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                if (got[b] == 0) continue;  // first of the two (or past the end): the partner finishes
                const uint32_t i = i0 + (uint32_t)b * 2u * 64u * W;
                const uint32_t ito = i / per, rem = i - ito * per;
                const uint32_t t = rem / (A.M * 16u), rem2 = rem - t * (A.M * 16u);
                const uint32_t sgi = j0 + ito * G;
                uint32_t mi = 0;
                for (uint32_t j = 1; j < A.nmat; ++j) mi = sgi >= A.mat[j].sg_begin ? j : mi;
                const StreamMat& Mt = A.mat[mi];
                const float plo = __uint_as_float(~(uint32_t)got[b]), phi = __uint_as_float(~(uint32_t)(got[b] >> 32));
                const float slo = ks == 0 ? o32[i] + plo : plo + o32[i];  // slice order
                const float shi = ks == 0 ? o32[i + 1] + phi : phi + o32[i + 1];
                const uint32_t col = ((sgi - Mt.sg_begin) * A.T + t) * 16u + (rem2 & 15u);
                *reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(Mt.y) + (rem2 >> 4) * Mt.N + col) =
                    pack2<DT>(slo, shi);
                __hip_atomic_store(A.slab + ent[b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        NF4_GSTAMP(5);
        NF4_GSTAMP(9);
        return;
    }
    for (uint32_t i = 2u * tid; i < mine * per; i += 2u * 64u * W) {  // column pairs
        const uint32_t ito = i / per, rem = i - ito * per;
        const uint32_t t = rem / (A.M * 16u), rem2 = rem - t * (A.M * 16u);
        const uint32_t sgi = j0 + ito * G;
        uint32_t mi = 0;
        for (uint32_t j = 1; j < A.nmat; ++j) mi = sgi >= A.mat[j].sg_begin ? j : mi;
        const StreamMat& Mt = A.mat[mi];
        const uint32_t gstrip = Mt.strip_begin + (sgi - Mt.sg_begin) * A.T + t;
        slab_put2(A.slab, slab_entry(ks, A.M, rem2 >> 4, A.ncols, gstrip * 16u + (rem2 & 15u)), o32[i], o32[i + 1]);
    }
    // (no wait for the entries' write acknowledgements: the reducer polls them)
    __syncthreads();
    for (uint32_t ito = wave; ito < mine; ito += W) {
        const uint32_t sgi = j0 + ito * G;
        uint32_t last = 0;
        if (lane == 0) last = splitk_ticket(&A.counters[sgi], KS);
        last = __builtin_amdgcn_readfirstlane(last);
        if (!last) continue;
        uint32_t mi = 0;
        for (uint32_t j = 1; j < A.nmat; ++j) mi = sgi >= A.mat[j].sg_begin ? j : mi;
        const StreamMat& Mt = A.mat[mi];
        const uint32_t s0 = (sgi - Mt.sg_begin) * A.T;  // first strip of the group within the weight
        const uint32_t col0 = (Mt.strip_begin + s0) * 16u;
        if (A.T == 4) splitk_reduce<DT, 64u>(A.slab, KS, A.M, A.ncols, col0, Mt.y, Mt.N, s0 * 16u, lane, A.counters);
        else if (A.T == 2) splitk_reduce<DT, 32u>(A.slab, KS, A.M, A.ncols, col0, Mt.y, Mt.N, s0 * 16u, lane, A.counters);
        else splitk_reduce<DT, 16u>(A.slab, KS, A.M, A.ncols, col0, Mt.y, Mt.N, s0 * 16u, lane, A.counters);
    }
    NF4_GSTAMP(5);
    }
    NF4_GSTAMP(9);
}


}  // namespace
