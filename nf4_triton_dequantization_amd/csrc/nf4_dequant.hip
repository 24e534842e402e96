// nf4_dequant.hip -- MI355X (gfx950 / CDNA4) NF4 double-dequantization kernels
// and the C ABI declared in include/nf4_dequant.h.
//
// What it replaces: the Triton kernel _nf4_dequantize_kernel_final
// (reference nf4_triton_dequantization/kernel_optimized.py:11-110) and its
// launcher _triton_dequantize_main (:142-205).  Semantics are the reference
// fallback's (_aggressive_pytorch_t4, :208-314), bit for bit; see
// oracle/nf4_oracle.c for the CPU restatement and DESIGN.md for the layout.
//
// Design (bandwidth-bound: 0.5 B in + 2 B out per element, no MFMA):
//  * "flat" kernel: whenever no 64-column block straddles a row (n % 64 == 0 and
//    the packed rows are dense) the packed weight is one byte stream.  A wave
//    owns a tile of 256*U packed bytes; lane l loads dword j at
//    tile + 256*j + 4*l, so each load instruction reads 256 contiguous bytes and
//    each of the U 16-byte output stores writes 1 KiB contiguous per wave:
//    every HBM line is written whole by one store instruction.  Loads and
//    stores are buffer instructions (range-checked: partial tiles need no
//    predicates), output stores are non-temporal (written once, streamed),
//    and a capped grid's wave loop is software-pipelined: the next tile's loads
//    are in flight while the current tile is decoded and stored.
//  * one lane per 64-element block computes the block's scale (absmax byte,
//    nested absmax, IEEE fp32 division by 127 -- never a reciprocal), and the
//    eight lanes that own the block's dwords fetch it with ds_bpermute.
//  * 16-bit outputs decode through a per-block table (round 5): the 8 lanes of a
//    64-element block round its 16 possible outputs (fp32 product, then
//    v_cvt_pk_{bf16,f16}_f32, round to nearest even) into 32 bytes of LDS, and every
//    output is one 16-bit lookup whose address is a single v_perm_b32; high nibble
//    -> even column.  fp32 output (quant_state.dtype = torch.float32) looks the code
//    up in the 16-entry LDS table and stores the product unrounded.
//  * the default grid gives every wave exactly one tile (tiles/4 workgroups), which it
//    runs straight through; only a grid capped through nf4_dequant_ref_cfg makes waves
//    walk several tiles in the software-pipelined loop.
//  * batched: up to NF4DQ_BATCH_MAX matrices per launch in the kernel
//    arguments; a wave finds its matrix by scanning scalar tile offsets.
//  * "chunk" kernels (round 5): any other shape (partial blocks, padded rows, odd n,
//    unaligned pointers) -- the flat tile with rows cut out of the stream and
//    one LDS table per scale block of the wave; the one-thread-per-byte "rows"
//    kernel only past their 32-bit index limits.
//  * "piece" kernels (round 6): of those, every row of >= 512 elements the chunk
//    kernel could not store whole (n % 8 != 0, a misaligned output or packed
//    weight, fp32 output), in OUTPUT order: 16-byte output pieces stored straight
//    from registers, the irregularity moved to the packed loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nf4_dequant.h"
#include "nf4_common.h"

namespace {

using namespace nf4dq;

enum Mode : int { kRef = 0, kSingle = 1, kBnb = 2, kBnbSingle = 3 };

// Kernel-argument image of one matrix on the flat path.
struct Desc {
    const uint32_t* packed;  // dense packed stream (4-byte aligned)
    const uint8_t* a1;       // uint8 absmax (ref, bnb)
    const float* a2;         // nested absmax (ref, bnb) or fp32 absmax (single modes)
    const float* code2;      // bnb nested code book (256 fp32)
    u32x4* out;              // 16-byte aligned output
    float offset;            // bnb offset
    uint32_t nbytes;         // packed bytes (multiple of 4)
    uint32_t tile_begin;     // first tile of this matrix within the launch
    uint32_t groups;         // ceil(bpr/4) (ref)
    FastDiv nb;              // ref: modulus of A1 index
    FastDiv n2;              // ref: modulus of A2 index; single: .d = row stride
    FastDiv bpr;             // blocks per row
    uint32_t blk_shift;      // log2(bytes per scale block)
    uint32_t blk2_shift;     // bnb: log2(blocksize2)
    uint32_t blk_base;       // scale blocks before this piece (a matrix above kPieceBytes is several pieces)
};

// Diagnostic build only (tools/Makefile `stamps`): per-wave s_memrealtime stamps of
// the flat kernel -- entry, first tile decoded and stored (its loads arrived), exit
// after its stores completed, tiles walked -- into a buffer set by nf4_dbg_set_stamps.
#ifndef NF4_FLAT_STAMPS
#define NF4_FLAT_STAMPS 0
#endif

template <int MAXB>
struct Batch {
    Desc d[MAXB];
    uint32_t count;
    uint32_t total_tiles;
#if NF4_FLAT_STAMPS
    unsigned long long* stamps;
#endif
};

#if NF4_FLAT_STAMPS
#define NF4_FSTAMP(slot_, val_)                                                                      \
    do {                                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                                           \
        if (lane == 0) bt.stamps[(blockIdx.x * kFlatWaves + (threadIdx.x >> 6)) * 4u + (slot_)] = (val_); \
        __builtin_amdgcn_sched_barrier(0);                                                           \
    } while (0)
#define NF4_FNOW() __builtin_amdgcn_s_memrealtime()
#else
#define NF4_FSTAMP(slot_, val_) \
    do {                        \
    } while (0)
#define NF4_FNOW() 0ull
#endif

// Scalar store of one output element (rows kernels).
template <int DT>
__device__ __forceinline__ void store1(void* out, int64_t i, float x) {
    if constexpr (DT == NF4DQ_BF16) {
        reinterpret_cast<__bf16*>(out)[i] = (__bf16)x;
    } else if constexpr (DT == NF4DQ_F16) {
        reinterpret_cast<_Float16*>(out)[i] = (_Float16)opaque(x);
    } else {
        reinterpret_cast<float*>(out)[i] = x;
    }
}

// Variant hooks of the flat kernel: the product values by default.  tools/dq_variants.hip
// redefines them to build A/B libraries (tools/_build/libnf4dq_dqv_<x>.so, timed in the
// HBM-streamed regime by tools/stream_probe.py / cache_ab.py --libs); nothing in the
// product sets them.  Hooks whose variants measured slower were removed after measurement
// (profiles/r05/README.md names them and the commits that still have them).
//   NF4_DQ_FLAT_WAVES   waves per workgroup of the flat kernel (4)
//   NF4_DQ_U            packed dwords per lane per tile (4: 1 KiB of packed bytes per wave)
//   NF4_DQ_AUX_STORE    cache-policy bits of the output stores (18 = sc1 + nt)
//   NF4_DQ_AUX_LOAD     cache-policy bits of the packed-weight loads (2 = nt)
//   NF4_DQ_SCALE_FIRST  1: a tile's absmax / nested-scale loads go out before its packed loads
//   NF4_DQ_SCALE_NT     1: the absmax / nested-scale gathers carry the nt policy too
//   NF4_DQ_DECODE       16-bit outputs: 1 (product) = per-block table of the 16 rounded
//                       outputs in LDS (tile_finish_tbl); 0 = code lookup per nibble + fp32
//                       multiply + rounding per output (rounds 1-4; fp32 output always takes
//                       this path).  HBM-streamed 4096^2 bf16: 7.33-7.36 us per launch vs
//                       7.62-7.65 (profiles/r05/dequant_decode_ab.jsonl)
//   NF4_DQ_SINGLE_FAST  1 (product): a wave with one tile skips the pipelined loop (next-tile
//                       loads, dropped-store burst); 7.33 -> 7.22 us per streamed 4096^2
//                       launch at K = 128 (profiles/r05/single_tile_fast_path_ab.jsonl)
//   NF4_DQ_ABL_NOSCALE  ablation (wrong results, tools only): no absmax / nested-absmax loads
#ifndef NF4_DQ_FLAT_WAVES
#define NF4_DQ_FLAT_WAVES 4
#endif
#ifndef NF4_DQ_U
#define NF4_DQ_U 4
#endif
#ifndef NF4_DQ_AUX_STORE
#define NF4_DQ_AUX_STORE 18
#endif
#ifndef NF4_DQ_AUX_LOAD
#define NF4_DQ_AUX_LOAD 2
#endif
#ifndef NF4_DQ_SCALE_FIRST
#define NF4_DQ_SCALE_FIRST 0
#endif
#ifndef NF4_DQ_SCALE_NT
#define NF4_DQ_SCALE_NT 0
#endif
#ifndef NF4_DQ_DECODE
#define NF4_DQ_DECODE 1
#endif
#ifndef NF4_DQ_SINGLE_FAST
#define NF4_DQ_SINGLE_FAST 1
#endif
#ifndef NF4_DQ_ABL_NOSCALE
#define NF4_DQ_ABL_NOSCALE 0
#endif



constexpr int kWg = 256;   // rows / bitsandbytes-bytes kernels: 4 waves per workgroup
constexpr int kFlatWaves = NF4_DQ_FLAT_WAVES;  // the flat kernel's workgroup
constexpr int kFlatWg = 64 * kFlatWaves;
constexpr int kU = NF4_DQ_U;  // packed dwords (fp32 output: words) per lane per tile

// Cache-policy bits of the buffer instructions (aux operand, gfx950 CPol):
// 2 = nt (streaming), 16 = sc1.  Output stores are sc1+nt: a write-once stream,
// not kept in the XCD L2 (+25-30 % over default-policy stores, profiles/r01/tune_sweep.log).
// Round 5, weights streamed from HBM: nt-only stores make the memory-system twin 2 %
// faster but the product 4-5 % slower at 4096^2 and 8192^2 alike (they interact with the
// scale gathers; profiles/r05/decode_store_variants_4096.jsonl, store_policy_large.jsonl).
constexpr int kAuxStore = NF4_DQ_AUX_STORE;
// Packed-weight loads are nt (streaming; round 4): a streamed model reads each weight
// once, from HBM.  With the default policy a 4096^2 launch whose weights come from
// HBM takes 7.95 us (66 %); with nt loads 7.46-7.49 us (70-71 %), the same whether or
// not the weights are still in the Infinity Cache (nt reads do not use it: the
// cache-warm figure becomes 7.45 instead of 6.86 us).  Sc0 / sc1 bits beside nt
// change nothing (profiles/r04/cache/dequant_variants_4096.jsonl).
constexpr int kAuxLoad = NF4_DQ_AUX_LOAD;

template <int DT>
constexpr uint32_t out_bytes_per_packed_byte() { return DT == NF4DQ_F32 ? 8u : 4u; }
// Packed bytes a lane loads per step j: 4 (-> 8 outputs = 16 B of fp16/bf16) or,
// for fp32 output, 2 (-> 4 outputs = 16 B).  Either way every lane stores 16 B
// per step and a wave store instruction covers 1 KiB contiguous.
template <int DT>
constexpr uint32_t lane_bytes() { return DT == NF4DQ_F32 ? 2u : 4u; }
template <int DT>
constexpr uint32_t tile_bytes() { return 64u * lane_bytes<DT>() * kU; }

// Raw inputs of one wave-tile, loaded ahead of use (software pipeline stage 1).
struct TileIn {
    uint32_t w[kU];  // packed dwords of this lane
    uint32_t a1;     // raw absmax byte of this lane's scale block (ref / bnb)
    float a2;        // nested absmax (ref / bnb) or fp32 absmax (single modes)
};

// Block index (within the whole matrix / stream) of this lane's scale block in tile `base`.
template <int DT>
__device__ __forceinline__ uint32_t tile_block(const Desc& D, uint32_t base, uint32_t lane) {
    constexpr uint32_t kTileBytes = tile_bytes<DT>();
    const uint32_t bsh = D.blk_shift;
    const uint32_t bpt = kTileBytes >> bsh;  // 0 when one block spans the tile
    uint32_t g = (base >> bsh) + (bpt ? (lane & (bpt - 1u)) : 0u);
    const uint32_t nblk = (D.nbytes + (1u << bsh) - 1u) >> bsh;
    g = g < nblk ? g : nblk - 1u;  // lanes past the end read a valid block; their stores drop
    return g + D.blk_base;
}

// Issue the loads of tile `base` (packed bytes) of matrix D.  Buffer loads
// outside the matrix return 0, so partial tiles need no predicates.
template <int DT, int MODE>
__device__ __forceinline__ TileIn tile_load(const Desc& D, __amdgpu_buffer_rsrc_t rp, uint32_t base, uint32_t lane) {
    constexpr uint32_t LB = lane_bytes<DT>();
    TileIn in;
    auto packed_loads = [&]() {
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            const uint32_t off = base + 64u * LB * j + LB * lane;
            if constexpr (LB == 4) {
                in.w[j] = __builtin_amdgcn_raw_buffer_load_b32(rp, off, 0, kAuxLoad);
            } else {
                in.w[j] = __builtin_amdgcn_raw_buffer_load_b16(rp, off, 0, kAuxLoad);
            }
        }
    };
    if constexpr (!NF4_DQ_SCALE_FIRST) packed_loads();
    const uint32_t g = tile_block<DT>(D, base, lane);
    if constexpr (NF4_DQ_ABL_NOSCALE) {
        in.a1 = g & 255u;
        in.a2 = 0.01f;
    } else if constexpr (MODE == kRef) {
        // (host-proven shortcuts for these indices -- one shift instead of the three
        // magic-number divisions -- measured no faster: the gathers issued earlier cost as
        // much as they save, profiles/r05/fast_index_ab.jsonl, gather_delay_variants.jsonl)
        const uint32_t r = fdiv(g, D.bpr);
        const uint32_t b = g - r * D.bpr.d;
        const uint8_t* pa1 = D.a1 + fmodu(g, D.nb);
        const float* pa2 = D.a2 + fmodu(r * D.groups + (b >> 2), D.n2);
        if constexpr (NF4_DQ_SCALE_NT) {
            in.a1 = __builtin_nontemporal_load(pa1);
            in.a2 = __builtin_nontemporal_load(pa2);
        } else {
            in.a1 = *pa1;
            in.a2 = *pa2;
        }
    } else if constexpr (MODE == kSingle) {
        const uint32_t r = fdiv(g, D.bpr);
        const uint32_t b = g - r * D.bpr.d;
        in.a2 = D.a2[r * D.n2.d + b];
    } else if constexpr (MODE == kBnb) {
        in.a1 = D.a1[g];
        in.a2 = D.a2[g >> D.blk2_shift];
    } else {
        in.a2 = D.a2[g];
    }
    if constexpr (NF4_DQ_SCALE_FIRST) packed_loads();
    return in;
}

// Stage 2: scale of this lane's block, ds_bpermute to the dword owners, decode,
// round, and kU 16-byte stores -- each wave store instruction writes 1 KiB
// contiguous; stores past the end of the matrix are dropped by the buffer range
// check.
template <int DT, int MODE>
__device__ __forceinline__ void tile_finish(const Desc& D, __amdgpu_buffer_rsrc_t ro, const float* lut,
                                            const TileIn& in, uint32_t base, uint32_t lane, const float* code2s) {
    float s;
    if constexpr (MODE == kRef) {
        s = ((float)in.a1 / 127.0f) * in.a2;  // IEEE division (:45, :270), then fp32 multiply
    } else if constexpr (MODE == kBnb) {
        // the 256-entry code from the workgroup's LDS copy: a global gather here
        // would wait on the absmax byte and then on L2 again, once per tile
        s = code2s[in.a1] * in.a2 + D.offset;
    } else {
        s = in.a2;
    }
    const uint32_t bsh = D.blk_shift;
    constexpr uint32_t kOB = out_bytes_per_packed_byte<DT>();
    constexpr uint32_t LB = lane_bytes<DT>();
#pragma unroll
    for (int j = 0; j < kU; ++j) {
        const uint32_t rel = 64u * LB * j + LB * lane;
        const float sj = __shfl(s, (int)(rel >> bsh), 64);
        const uint32_t w = in.w[j];
        const uint32_t hi4 = (w >> 2) & 0x3C3C3C3Cu;
        const uint32_t lo4 = (w << 2) & 0x3C3C3C3Cu;
        const char* t = reinterpret_cast<const char*>(lut);
        float v[2 * LB];
#pragma unroll
        for (int k = 0; k < (int)LB; ++k) {
            v[2 * k] = *reinterpret_cast<const float*>(t + ((hi4 >> (8 * k)) & 0xFFu)) * sj;
            v[2 * k + 1] = *reinterpret_cast<const float*>(t + ((lo4 >> (8 * k)) & 0xFFu)) * sj;
        }
        const uint32_t ob = (base + rel) * kOB;
        if constexpr (DT == NF4DQ_F32) {
            u32x4 o = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
            __builtin_amdgcn_raw_buffer_store_b128(o, ro, ob, 0, kAuxStore);
        } else {
            u32x4 o = {pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]), pack2<DT>(v[6], v[7])};
            __builtin_amdgcn_raw_buffer_store_b128(o, ro, ob, 0, kAuxStore);
        }
    }
}

// Stage 2, table decode (NF4_DQ_DECODE == 1, 16-bit outputs).  Dword j of lane l lies
// in block 8j + l/8 of the tile, shared by the 8 lanes of group l/8; lane 8g + k rounds
// the block's outputs for codes 2k and 2k+1 (the same fp32 products and RNE as the
// per-nibble path) into dword k of the group's 16-entry table, at LDS byte tb + 4k
// (tb = the wave's region + 256 g: byte 0 of tb is zero).  An output is then the 16-bit
// entry at tb + 2 * code, and 2 * code is a byte of (w >> 3) & 0x1E1E1E1E (high nibbles)
// or (w << 1) & 0x1E1E1E1E (low nibbles): v_perm_b32 moves that byte into tb's byte 0,
// one instruction per address.  The 8 lanes of a group write their table before any of
// them reads it in program order, and a wave's LDS accesses complete in order, so no
// barrier; the next dword's table reuses the region after this one's reads.
typedef uint16_t __attribute__((may_alias)) u16_alias;  // table entries are written as dwords
typedef uint32_t __attribute__((may_alias)) u32_alias;
typedef uint32_t u32x4_alias __attribute__((ext_vector_type(4), may_alias));

struct TblCtx {
    char* tbl;    // LDS base of the workgroup's tables
    uint32_t tb;  // this lane's group table offset (multiple of 256)
    f32x2 c01;    // NF4 codes 2k, 2k+1 of this lane (k = lane & 7)
};

template <int DT, int MODE>
__device__ __forceinline__ void tile_finish_tbl(const Desc& D, __amdgpu_buffer_rsrc_t ro, const TileIn& in,
                                                uint32_t base, uint32_t lane, const float* code2s,
                                                const TblCtx& c) {
    float s;
    if constexpr (MODE == kRef) {
        s = ((float)in.a1 / 127.0f) * in.a2;  // IEEE division (:45, :270), then fp32 multiply
    } else if constexpr (MODE == kBnb) {
        s = code2s[in.a1] * in.a2 + D.offset;
    } else {
        s = in.a2;
    }
    const uint32_t bsh = D.blk_shift;
    const uint32_t k = lane & 7u;
#pragma unroll
    for (int j = 0; j < kU; ++j) {
        const uint32_t rel = 256u * j + 4u * lane;
        const float sj = __shfl(s, (int)(rel >> bsh), 64);
        *reinterpret_cast<u32_alias*>(c.tbl + c.tb + 4u * k) = pack2<DT>(c.c01.x * sj, c.c01.y * sj);
        const uint32_t w = in.w[j];
        const uint32_t hb = (w >> 3) & 0x1E1E1E1Eu;
        const uint32_t lb = (w << 1) & 0x1E1E1E1Eu;
        uint32_t o[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t ah = __builtin_amdgcn_perm(hb, c.tb, 0x03020104u + b);
            const uint32_t al = __builtin_amdgcn_perm(lb, c.tb, 0x03020104u + b);
            const uint32_t vh = *reinterpret_cast<const u16_alias*>(c.tbl + ah);
            const uint32_t vl = *reinterpret_cast<const u16_alias*>(c.tbl + al);
            o[b] = vh | (vl << 16);
        }
        const u32x4 ov = {o[0], o[1], o[2], o[3]};
        __builtin_amdgcn_raw_buffer_store_b128(ov, ro, (base + rel) * 4u, 0, kAuxStore);
    }
}

template <int MAXB>
__device__ __forceinline__ uint32_t find_matrix(const Batch<MAXB>& bt, uint32_t t, uint32_t k) {
    if constexpr (MAXB > 1) {
        while (k + 1 < bt.count && t >= bt.d[k + 1].tile_begin) ++k;
    }
    return k;
}

// Position of a wave in the launch: tile t of the launch = tile of matrix k
// starting at packed byte `base`.
struct Cursor {
    uint32_t t, k, base;
    bool valid;
};

template <int DT, int MAXB>
__device__ __forceinline__ Cursor cursor_at(const Batch<MAXB>& bt, uint32_t t, uint32_t k_hint) {
    constexpr uint32_t kTileBytes = tile_bytes<DT>();
    Cursor c;
    c.t = t;
    c.valid = t < bt.total_tiles;
    c.k = c.valid ? find_matrix(bt, t, k_hint) : k_hint;
    // past the end: an offset beyond every buffer range (loads return 0, stores drop)
    c.base = c.valid ? (t - bt.d[c.k].tile_begin) * kTileBytes : 0xFFFFF000u;
    return c;
}

template <int DT, int MAXB>
__device__ __forceinline__ void make_rsrcs(const Batch<MAXB>& bt, uint32_t k, __amdgpu_buffer_rsrc_t& rp,
                                           __amdgpu_buffer_rsrc_t& ro) {
    constexpr uint32_t kOB = out_bytes_per_packed_byte<DT>();
    rp = __builtin_amdgcn_make_buffer_rsrc((void*)bt.d[k].packed, 0, bt.d[k].nbytes, kRsrcFlags);
    ro = __builtin_amdgcn_make_buffer_rsrc((void*)bt.d[k].out, 0, bt.d[k].nbytes * kOB, kRsrcFlags);
}

// The flat kernel.  Wave t owns tile t; with the default grid that is its only tile and
// it runs it straight through.  Under a capped grid (nf4_dequant_ref_cfg) waves walk
// tiles t, t + nwaves, ... in a loop unrolled by two with the tiles in two register
// sets (A, B), so that tile i+1's loads are in flight while tile i is decoded and
// stored, with no register copies (a copy would force a wait on the loads it copies).
template <int DT, int MODE, int MAXB>
__global__ __launch_bounds__(kFlatWg) void nf4_flat_kernel(const Batch<MAXB> bt) {
    __shared__ __attribute__((aligned(16))) float lut[16];
    __shared__ __attribute__((aligned(16))) float code2s[MODE == kBnb ? 256 : 1];  // bitsandbytes code (every piece's)
    constexpr bool kTbl = NF4_DQ_DECODE == 1 && DT != NF4DQ_F32;
    __shared__ __attribute__((aligned(256))) char tbl[kTbl ? kFlatWaves * 2048 : 4];  // 8 block tables per wave
    const uint32_t lane = threadIdx.x & 63u;
#if NF4_FLAT_STAMPS
    const unsigned long long t_entry = NF4_FNOW();
    unsigned long long tiles_done = 0;
#endif
    const uint32_t t0 = __builtin_amdgcn_readfirstlane(blockIdx.x * kFlatWaves + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * kFlatWaves;

    // First tile's loads go out before anything else (a wave without work
    // issues them past the buffer range: no traffic); the LUT write and the
    // barrier then overlap their latency.
    // bitsandbytes mode: each thread's word of the 256-entry nested code goes out ahead of
    // the tile's loads, so the wait before the barrier below covers only it (after them,
    // the wait covered the tile's loads too: 7.48 -> 7.44 us per streamed 4096^2 launch,
    // profiles/r05/bnb_mode_code_early.jsonl)
    float c2w = 0.0f;
    if constexpr (MODE == kBnb) c2w = bt.d[0].code2[threadIdx.x & 255u];
    Cursor ca = cursor_at<DT>(bt, t0, 0u);
    __amdgpu_buffer_rsrc_t rpa, roa;
    make_rsrcs<DT>(bt, ca.k, rpa, roa);
    TileIn A = tile_load<DT, MODE>(bt.d[ca.k], rpa, ca.base, lane);
    // Does this wave walk more than one tile?  (wave-uniform; with the default, uncapped
    // grid every wave has exactly one.)  A one-tile wave skips the pipelined loop: no
    // loads of a next tile past the end and no dropped store burst below -- half of its
    // vector-memory instructions otherwise.
    const bool multi = !NF4_DQ_SINGLE_FAST || ca.t + nwaves < bt.total_tiles;
    // Out-of-range (dropped) stores with the loop body's count: loop entry then
    // looks like the back edge to hipcc's waitcnt pass ([loads][stores]), so the
    // in-loop waits count past the previous tile's stores instead of draining them.
    if (multi) {
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < kU; ++j) __builtin_amdgcn_raw_buffer_store_b128(z, roa, 0xFFFFF000u + 16u * j, 0, kAuxStore);
    }
    // (the table decode could take its two codes from immediates and skip this table and
    // the barrier: measured 8 % slower, profiles/r05/nolut_scalefirst_variants.jsonl)
    write_lut(lut);
    if constexpr (MODE == kBnb) {  // every piece of a bitsandbytes stream carries the same code
        // (one 16-B load per lane of wave 0 ahead of everything measured slower, and no
        // table at all only 0.6 % faster: profiles/r05/bnb_mode_code_table.jsonl)
        if constexpr (kFlatWg >= 256) {
            if (threadIdx.x < 256u) code2s[threadIdx.x] = c2w;
        } else {  // (narrower workgroups of the A/B builds)
            for (uint32_t i = threadIdx.x; i < 256u; i += kFlatWg) code2s[i] = bt.d[0].code2[i];
        }
    }
    __syncthreads();
    TblCtx tc{};
    if constexpr (kTbl) {
        tc.tbl = tbl;
        tc.tb = ((threadIdx.x >> 6) << 11) + ((lane >> 3) << 8);
        tc.c01 = *reinterpret_cast<const f32x2*>(lut + 2u * (lane & 7u));
    }
    if (!ca.valid) {
        NF4_FSTAMP(0, t_entry);
        NF4_FSTAMP(1, 0ull);
        NF4_FSTAMP(2, NF4_FNOW());
        NF4_FSTAMP(3, 0ull);
        return;
    }
    if (!multi) {
        if constexpr (kTbl) tile_finish_tbl<DT, MODE>(bt.d[ca.k], roa, A, ca.base, lane, code2s, tc);
        else tile_finish<DT, MODE>(bt.d[ca.k], roa, lut, A, ca.base, lane, code2s);
#if NF4_FLAT_STAMPS
        NF4_FSTAMP(1, NF4_FNOW());
        __builtin_amdgcn_s_waitcnt(0);
        NF4_FSTAMP(0, t_entry);
        NF4_FSTAMP(2, NF4_FNOW());
        NF4_FSTAMP(3, 1ull);
#endif
        return;
    }
    while (true) {
        const Cursor cb = cursor_at<DT>(bt, ca.t + nwaves, ca.k);
        __amdgpu_buffer_rsrc_t rpb = rpa, rob = roa;
        if (MAXB > 1 && cb.k != ca.k) make_rsrcs<DT>(bt, cb.k, rpb, rob);
        TileIn B = tile_load<DT, MODE>(bt.d[cb.k], rpb, cb.base, lane);
        if constexpr (kTbl) tile_finish_tbl<DT, MODE>(bt.d[ca.k], roa, A, ca.base, lane, code2s, tc);
        else tile_finish<DT, MODE>(bt.d[ca.k], roa, lut, A, ca.base, lane, code2s);
#if NF4_FLAT_STAMPS
        if (tiles_done == 0) NF4_FSTAMP(1, NF4_FNOW());
        ++tiles_done;
#endif
        if (!cb.valid) break;

        const Cursor cn = cursor_at<DT>(bt, cb.t + nwaves, cb.k);
        __amdgpu_buffer_rsrc_t rpn = rpb, ron = rob;
        if (MAXB > 1 && cn.k != cb.k) make_rsrcs<DT>(bt, cn.k, rpn, ron);
        A = tile_load<DT, MODE>(bt.d[cn.k], rpn, cn.base, lane);
        if constexpr (kTbl) tile_finish_tbl<DT, MODE>(bt.d[cb.k], rob, B, cb.base, lane, code2s, tc);
        else tile_finish<DT, MODE>(bt.d[cb.k], rob, lut, B, cb.base, lane, code2s);
#if NF4_FLAT_STAMPS
        ++tiles_done;
#endif
        if (!cn.valid) break;
        ca = cn;
        rpa = rpn;
        roa = ron;
    }
#if NF4_FLAT_STAMPS
    __builtin_amdgcn_s_waitcnt(0);  // every load and store of this wave complete
    NF4_FSTAMP(0, t_entry);
    NF4_FSTAMP(2, NF4_FNOW());
    NF4_FSTAMP(3, tiles_done);
#endif
}

// Any shape, reference / single-quant semantics: one thread per packed byte.  Only for
// matrices past the chunk kernel's 32-bit index limits (below) or when a tuning call
// asks for it (NF4DQ_CFG_ROWS).
struct RowsArgs {
    const uint8_t* packed;
    const uint8_t* a1;
    const float* a2;
    void* out;
    int64_t m, n, stride, cols_b;  // cols_b = ceil(n/2) packed bytes used per row
    int64_t nb, n2, bpr, groups, rs;
};

template <int DT, int MODE>
__global__ __launch_bounds__(kWg) void nf4_rows_kernel(const RowsArgs A) {
    __shared__ __attribute__((aligned(16))) float lut[16];
    write_lut(lut);
    __syncthreads();
    const int64_t total = A.m * A.cols_b;
    for (int64_t i = (int64_t)blockIdx.x * kWg + threadIdx.x; i < total; i += (int64_t)gridDim.x * kWg) {
        const int64_t r = i / A.cols_b;
        const int64_t j = i - r * A.cols_b;
        const int64_t b = j >> 5;
        float s;
        if constexpr (MODE == kRef) {
            const float q = (float)A.a1[(r * A.bpr + b) % A.nb];
            s = (q / 127.0f) * A.a2[(r * A.groups + (b >> 2)) % A.n2];
        } else {
            s = A.a2[r * A.rs + b];
        }
        const uint32_t byte = A.packed[r * A.stride + j];
        const int64_t c = 2 * j;
        store1<DT>(A.out, r * A.n + c, lut[byte >> 4] * s);
        if (c + 1 < A.n) store1<DT>(A.out, r * A.n + c + 1, lut[byte & 15u] * s);
    }
}

// The chunk kernels (round 5): every shape the flat kernel does not take -- n % 64 != 0
// (rows end in a partial 64-column block), padded rows, unaligned pointers -- with
// reference / single-quant semantics.  Each row's packed bytes are cut into 4-byte
// chunks (L = ceil(ceil(n/2) / 4) per row); chunk c = r * L + q holds columns 8q .. 8q+7
// of row r, all inside 64-column block q / 8.  A wave owns 256 consecutive chunks, lane l
// chunk 64 j + l at step j -- the flat kernel's tile with rows cut out of the stream.
// Blocks no longer line up with groups of 8 lanes, but the wave's blocks are consecutive
// (block g = r * bpr + q / 8 steps by one per 8 chunks, and from a row's last block to the
// next row's first): lane i gathers block g0 + i's scale and rounds its 16 outputs into a
// table of the wave's (one per block), and every output is a table lookup.
//  * nf4_chunk_dense_kernel: 16-bit output, n % 8 == 0 and packed rows of exactly 4 L
//    bytes (the usual odd-width weight): chunk c is packed bytes 4c.. and output elements
//    8c.., the flat kernel's stream, so loads and stores need no row arithmetic.
//    4096 x 4080 bf16: 7.49 us = 70 % of 8 TB/s (flat 4096^2 7.36 on the same box; the
//    per-byte kernel 33.5), profiles/r05/chunk/s37_chunk_ab_dense_form.jsonl.
//  * nf4_chunk_kernel: the rest.  The buffer bases are the wave's first row / output
//    element (scalar 64-bit), so only offsets within one wave's span are 32-bit; rows of
//    >= 64 chunks advance their indices by additions, shorter rows divide per step (and
//    gather per lane when the wave spans more than 64 blocks).  16-bit outputs that cannot
//    take one 16-byte store per chunk (n % 8 != 0, or the output off 16-byte alignment)
//    are staged through LDS and written as aligned 16-byte pieces (store16 / flush16):
//    17.9 / 15.3 us at 4096 x 4090 / 4095 (28.6 us at 4095 storing from the lanes).
struct ChunkArgs {
    const uint8_t* packed;
    const uint8_t* a1;
    const float* a2;
    void* out;
    uint64_t packed_len;  // bytes (the load range)
    uint64_t out_elems;   // m * n
    uint32_t stride;      // packed bytes per row
    uint32_t n;           // columns
    uint32_t chunks;      // m * L
    FastDiv L;            // chunks per row
    FastDiv bpr;          // 64-column blocks per row
    uint32_t groups;      // ceil(bpr / 4)
    FastDiv nb, n2;       // ref: moduli of the absmax / nested-absmax indices
    uint32_t rs;          // single: absmax per row
};

constexpr uint32_t kDrop = 0xFFFFFFF0u;  // an offset past every range: load 0 / store dropped
// Stores narrower than 16 bytes (fp32 elements of odd widths, the end pieces of a staged
// span) use the default policy, so that the L2 merges a line's pieces before it goes to
// HBM: streamed (nt) partial-line writes made odd-n matrices 5x slower still (s34, s35).
constexpr int kAuxPiece = 0;
// The general form's packed loads take the default policy too: a padded row's 256-byte
// load instructions straddle three lines, each shared with the next instruction, and nt
// lines are not kept for it (padded 4096^2: 9.99 -> 9.61 us, profiles/r05/chunk/s45).
// A wave's staged 16-bit span: 2048 elements + 7 of misalignment, then one dummy element
// (past-n elements of a partial chunk), rounded to 16 bytes.
constexpr uint32_t kStageBytes = 4128;
constexpr uint32_t kStageDummy = 4112;

inline __device__ uint32_t range32(uint64_t v) { return v > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)v; }

// a * b kept apart from the add that follows it: fused, hipcc emits a 64-bit multiply-add
// whose (ignored) high addend can be any register -- once a packed load's destination, so
// the scale gathers waited for that load (+1 us per launch).
inline __device__ uint32_t opaque_mul(uint32_t a, uint32_t b) {
    uint32_t r = a * b;
    asm("" : "+v"(r));
    return r;
}

// Block-table decode of one wave's 4 steps (16-bit output): lane i has rounded the 16
// outputs of block g0 + i (fp32 products and RNE, as everywhere) into 32 bytes at the
// wave's LDS region + 32 i.  Output (t = block - g0, code) is the 16-bit entry at region +
// 256 (t >> 3) + 32 (t & 7) + 2 code: the low byte is the code byte (2 code, from (w >> 3)
// or (w << 1) & 0x1E) ORed with 32 (t & 7) in every byte lane, and v_perm_b32 drops it
// below region + 256 (t >> 3) -- one instruction per address, as in the flat kernel, and
// no ds_bpermute of the scale.
template <int DT>
__device__ __forceinline__ void chunk_table_build(char* ctbl, uint32_t region, uint32_t lane, float sb) {
    uint32_t e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        e[k] = pack2<DT>(__uint_as_float(kNf4Bits[2 * k]) * sb, __uint_as_float(kNf4Bits[2 * k + 1]) * sb);
    u32x4_alias* dst = reinterpret_cast<u32x4_alias*>(ctbl + region + 32u * lane);
    dst[0] = u32x4{e[0], e[1], e[2], e[3]};
    dst[1] = u32x4{e[4], e[5], e[6], e[7]};
}

__device__ __forceinline__ void chunk_table_decode(const char* ctbl, uint32_t region, uint32_t w, uint32_t t,
                                                   uint32_t (&p)[4]) {
    t &= 63u;  // (lanes past the end: any table; their stores drop)
    const uint32_t base = region + ((t >> 3) << 8);
    const uint32_t rep = __builtin_amdgcn_perm(0u, (t & 7u) << 5, 0x00000000u);  // the byte in every lane
    const uint32_t hb = ((w >> 3) & 0x1E1E1E1Eu) | rep;
    const uint32_t lb = ((w << 1) & 0x1E1E1E1Eu) | rep;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t ah = __builtin_amdgcn_perm(hb, base, 0x03020104u + b);
        const uint32_t al = __builtin_amdgcn_perm(lb, base, 0x03020104u + b);
        const uint32_t vh = *reinterpret_cast<const u16_alias*>(ctbl + ah);
        const uint32_t vl = *reinterpret_cast<const u16_alias*>(ctbl + al);
        p[b] = vh | (vl << 16);
    }
}

// The chunk kernel's dense form: 16-bit output, n % 8 == 0, packed rows of exactly 4 L
// bytes, rows of >= 64 chunks, < 2 GiB each way.  Chunk c is then packed bytes 4c .. 4c+3
// and output elements 8c .. 8c+7 -- the flat kernel's stream -- so the loads go out first
// with no row arithmetic, the stores need none either, and only the scale blocks
// (r * bpr + q / 8) follow the rows.
template <int DT, int MODE>
__global__ __launch_bounds__(kWg) void nf4_chunk_dense_kernel(const ChunkArgs A) {
    __shared__ __attribute__((aligned(256))) char ctbl[4 * 2048];  // 64 block tables per wave
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cw = __builtin_amdgcn_readfirstlane((blockIdx.x * 4u + (threadIdx.x >> 6)) * 256u);
    const __amdgpu_buffer_rsrc_t rp =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.packed, 0, (uint32_t)A.packed_len, kRsrcFlags);
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(A.out, 0, (uint32_t)(A.out_elems * 2u), kRsrcFlags);
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)  // (past the end: out of range, no traffic)
        w[j] = __builtin_amdgcn_raw_buffer_load_b32(rp, 4u * (cw + 64u * j + lane), 0, kAuxLoad);
    __builtin_amdgcn_sched_barrier(0);  // (the scheduler would hoist the scale gathers above them)
    // The blocks of the wave's 256 chunks are consecutive and at most 38 (rows >= 64 chunks):
    // lane i gathers block g0 + i's scale (cf. the general form below).
    const uint32_t cw0 = min(cw, A.chunks - 1u);  // (a wave wholly past the end: cf. nf4_chunk_kernel)
    const uint32_t r0 = fdiv(cw0, A.L);
    const uint32_t q0 = cw0 - r0 * A.L.d;
    const uint32_t cl = min(cw + 255u, A.chunks - 1u);
    const uint32_t rl = fdiv(cl, A.L);
    const uint32_t g0 = r0 * A.bpr.d + (q0 >> 3);
    const uint32_t gl = rl * A.bpr.d + ((cl - rl * A.L.d) >> 3);
    float sb;
    {
        const uint32_t g = min(g0 + lane, gl);
        const uint32_t r = fdiv(g, A.bpr);
        const uint32_t b = g - r * A.bpr.d;
        if constexpr (MODE == kRef) {
            const float q8 = (float)A.a1[fmodu(g, A.nb)];
            sb = (q8 / 127.0f) * A.a2[fmodu(opaque_mul(r, A.groups) + (b >> 2), A.n2)];  // IEEE division (:45, :270)
        } else {
            sb = A.a2[opaque_mul(r, A.rs) + b];
        }
    }
    uint32_t gsel[4];
    {
        uint32_t q = q0 + lane;
        const bool wrap = q >= A.L.d;
        q = wrap ? q - A.L.d : q;
        uint32_t gr = (wrap ? A.bpr.d : 0u) + r0 * A.bpr.d - g0;  // r * bpr - g0
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j) {
                q += 64u;
                const bool wj = q >= A.L.d;
                q = wj ? q - A.L.d : q;
                gr += wj ? A.bpr.d : 0u;
            }
            gsel[j] = gr + (q >> 3);
        }
    }
    const uint32_t region = (threadIdx.x >> 6) << 11;
    chunk_table_build<DT>(ctbl, region, lane, sb);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t p[4];
        chunk_table_decode(ctbl, region, w[j], gsel[j], p);
        const u32x4 o = {p[0], p[1], p[2], p[3]};
        __builtin_amdgcn_raw_buffer_store_b128(o, ro, 16u * (cw + 64u * j + lane), 0, kAuxStore);
    }
}

// LW: 4 = dword loads (packed and stride 4-byte aligned), 1 = pairs of aligned dword loads
// joined with v_alignbyte (any alignment).
// SW: 16 = whole-chunk 16-byte stores (16-bit output: n % 8 == 0; fp32: n % 4 == 0, two
// per chunk; output 16-byte aligned); 4 = anything else: 16-bit outputs staged through
// LDS, fp32 outputs stored one element at a time.
template <int DT, int MODE, int LW, int SW>
__global__ __launch_bounds__(kWg) void nf4_chunk_kernel(const ChunkArgs A) {
    __shared__ __attribute__((aligned(16))) float lut[16];
    __shared__ __attribute__((aligned(256))) char ctbl[DT == NF4DQ_F32 ? 4 : 4 * 2048];  // 64 block tables per wave
    __shared__ __attribute__((aligned(16))) char stage[DT != NF4DQ_F32 && SW != 16 ? 4 * kStageBytes : 16];
    constexpr uint32_t kOB = DT == NF4DQ_F32 ? 4u : 2u;  // output bytes per element
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cw = __builtin_amdgcn_readfirstlane((blockIdx.x * 4u + (threadIdx.x >> 6)) * 256u);
    // A wave of the last workgroup can lie wholly past the end; its row base is clamped to
    // the last chunk's, so that the row indices every lane forms (scale gathers included)
    // stay inside the matrix -- its loads and stores are all out of range anyway.
    const uint32_t cw0 = min(cw, A.chunks - 1u);
    const uint32_t r0 = fdiv(cw0, A.L);
    const uint32_t q0 = cw0 - r0 * A.L.d;
    const uint64_t pb = (uint64_t)r0 * A.stride;
    // LW == 1 (a packed row start off 4-byte alignment): the buffer starts at the dword
    // holding the wave's first byte and ends at the dword holding the weight's last, and a
    // chunk is the two dwords around it joined with v_alignbyte_b32 -- 2 loads per chunk
    // instead of 4 byte loads.  The at most 3 bytes read before / after the weight lie in
    // the same dword, hence the same page, as its first / last byte.
    const uintptr_t pw = (uintptr_t)(A.packed + pb);
    const uint32_t kb = LW == 4 ? 0u : (uint32_t)(pw & 3u);
    const uint64_t plen = LW == 4 ? A.packed_len - pb : ((A.packed_len - pb + kb + 3u) & ~uint64_t(3));
    const __amdgpu_buffer_rsrc_t rp =
        __builtin_amdgcn_make_buffer_rsrc((void*)(pw - kb), 0, range32(plen), kRsrcFlags);
    auto load_chunk = [&](uint32_t po) -> uint32_t {
        if constexpr (LW == 4) {
            return __builtin_amdgcn_raw_buffer_load_b32(rp, po, 0, 0);  // (see kAuxPiece)
        } else {
            const uint32_t a = po == kDrop ? kDrop : po + kb;  // byte offset from the aligned base
            const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rp, a & ~3u, 0, 0);
            const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rp, (a & ~3u) + 4u, 0, 0);
            return __builtin_amdgcn_alignbyte(hi, lo, a & 3u);
        }
    };
    // The blocks of the wave's chunks are consecutive (block g = r * bpr + q / 8 steps by one
    // per 8 chunks, and from a row's last block to the next row's first): when they number
    // at most 64, lane i gathers block g0 + i's scale once and the lanes fetch theirs with
    // ds_bpermute, as in the flat kernel; a wider span (rows of a few chunks) gathers per lane.
    const uint32_t g0 = r0 * A.bpr.d + (q0 >> 3);
    uint32_t gl = 0;
    bool shared = false;
    auto span_blocks = [&]() {  // (formed after the loads are out: nothing before them needs it)
        const uint32_t cl = min(cw + 255u, A.chunks - 1u);
        const uint32_t rl = fdiv(cl, A.L);
        gl = rl * A.bpr.d + ((cl - rl * A.L.d) >> 3);
        shared = gl - g0 < 64u;
    };
    uint32_t w[4], rel[4], col[4], gsel[4];
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    uint32_t ga1 = 0;
    float ga2 = 0.0f;
    auto gather = [&]() {  // (after the packed loads are out, as in the flat kernel)
        if (shared) {
            const uint32_t g = min(g0 + lane, gl);
            const uint32_t r = fdiv(g, A.bpr);
            const uint32_t b = g - r * A.bpr.d;
            if constexpr (MODE == kRef) {
                ga1 = A.a1[fmodu(g, A.nb)];
                ga2 = A.a2[fmodu(opaque_mul(r, A.groups) + (b >> 2), A.n2)];
            } else {
                ga2 = A.a2[opaque_mul(r, A.rs) + b];
            }
        }
    };
    if (A.L.d >= 64u) {
        // Rows of >= 64 chunks (n >= 505): the wave touches at most 6 rows and 38 blocks
        // (shared scales), and step j+1's chunk is step j's + 64, at most one row further,
        // so every index advances by additions -- no division or multiply per step.
        uint32_t qj[4], dr[4];  // each step's chunk within its row, and rows past r0
        {
            uint32_t q = q0 + lane, d = 0, pr = 0;  // pr = (r - r0) * stride
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (j) q += 64u;
                const bool wrap = q >= A.L.d;
                q = wrap ? q - A.L.d : q;
                d += wrap ? 1u : 0u;
                pr += wrap ? A.stride : 0u;
                qj[j] = q;
                dr[j] = d;
                w[j] = load_chunk(cw + 64u * j + lane < A.chunks ? pr + 4u * q : kDrop);
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // (the loads first; everything below waits for them anyway)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool ok = cw + 64u * j + lane < A.chunks;
            col[j] = ok ? 8u * qj[j] : 0x7FFFFFF0u;  // past n (< 2^28) for every piece of a chunk past the end
            rel[j] = dr[j] * A.n + 8u * qj[j] - 8u * q0;
            gsel[j] = dr[j] * A.bpr.d + (qj[j] >> 3) - (q0 >> 3);
        }
    } else {
        // (indices first, then the loads, then any per-lane gathers; see opaque_mul)
        uint32_t po[4], pa1[4], pa2[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t c = cw + 64u * j + lane;
            const bool ok = c < A.chunks;
            const uint32_t r = ok ? fdiv(c, A.L) : r0;
            const uint32_t q = ok ? c - r * A.L.d : q0;
            po[j] = ok ? (r - r0) * A.stride + 4u * q : kDrop;
            col[j] = ok ? 8u * q : 0x7FFFFFF0u;
            rel[j] = (r - r0) * A.n + 8u * q - 8u * q0;
            gsel[j] = r * A.bpr.d + (q >> 3) - g0;
            const uint32_t b = q >> 3;
            if constexpr (MODE == kRef) {
                pa1[j] = fmodu(r * A.bpr.d + b, A.nb);
                pa2[j] = fmodu(opaque_mul(r, A.groups) + (b >> 2), A.n2);
            } else {
                pa1[j] = 0;
                pa2[j] = opaque_mul(r, A.rs) + b;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = load_chunk(po[j]);
        __builtin_amdgcn_sched_barrier(0);
        span_blocks();
        if (!shared) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if constexpr (MODE == kRef) s[j] = ((float)A.a1[pa1[j]] / 127.0f) * A.a2[pa2[j]];
                else s[j] = A.a2[pa2[j]];
            }
        }
    }
    if (A.L.d >= 64u) span_blocks();
    gather();  // (after the packed loads are out, as in the flat kernel)
    const uint64_t e0 = (uint64_t)r0 * A.n + 8ull * q0;  // the wave's first output element
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((char*)A.out + e0 * kOB), 0, range32((A.out_elems - e0) * kOB), kRsrcFlags);
    float sb = 0.0f;
    if constexpr (MODE == kRef) sb = ((float)ga1 / 127.0f) * ga2;  // IEEE division (:45, :270)
    else sb = ga2;
    // Narrow 16-bit outputs (n % 8 != 0, or the output off 16-byte alignment) go through
    // LDS.  The wave's outputs are one contiguous span of the output (a row's last, partial
    // chunk is followed by the next row's first), so each lane drops its chunk's valid
    // elements into a copy of the span shifted by the output's misalignment `sa`, and the
    // wave then writes the span as 16-byte pieces aligned in the output: whole pieces with
    // one 16-byte store each, the (at most two) pieces at the span's ends element by element,
    // since a neighbouring wave owns the rest of them.  (Storing 4- or 2-byte pieces
    // straight from the lanes took 20.8 / 28.6 us at 4096 x 4090 / 4095.)
    const uint32_t sbase = (threadIdx.x >> 6) * kStageBytes;
    const uint32_t sa = (uint32_t)(((uintptr_t)A.out >> 1) + e0) & 7u;
    auto store16 = [&](int j, const uint32_t (&p)[4]) {  // one chunk of 16-bit outputs
        if constexpr (SW == 16) {
            const u32x4 o = {p[0], p[1], p[2], p[3]};
            __builtin_amdgcn_raw_buffer_store_b128(o, ro, col[j] < A.n ? rel[j] * 2u : kDrop, 0, kAuxStore);
        } else {
            // All 8 elements go to the stage at 2 (rel + sa) + 2 i, past-n ones included (round 6:
            // one address per chunk instead of a compare + select per element).  A row's last,
            // partial chunk thus writes its past-n elements onto the first slots of the chunks
            // that follow it in the span; the rightful element of such a slot always has a
            // SMALLER index i in its own chunk than the past-n element that lands on it, and every
            // lane writes its elements from i = 7 down to 0, so the rightful one is written last
            // (the chunk after lane 63's is lane 0's at step j + 1: later in program order too).
            // The slack past the span's end covers the last chunk's past-n elements; chunks past
            // the end of the matrix write to the dummy slots.
            const bool ok = cw + 64u * (uint32_t)j + lane < A.chunks;
            char* a = stage + sbase + (ok ? 2u * (rel[j] + sa) : kStageDummy);
            // (the compiler barrier keeps the 8 stores apart: merged into one unaligned
            // ds_write_b128, a past-n element and the slot's rightful one would be written by
            // two lanes of the same instruction, in no defined order)
#pragma unroll
            for (int i = 7; i >= 0; --i) {
                reinterpret_cast<u16_alias*>(a)[i] = (uint16_t)(p[i >> 1] >> (16 * (i & 1)));
                asm volatile("" ::: "memory");
            }
        }
    };
    // The staged form's span: its length in elements and its first / last 128-byte line.
    // Whole 16-byte pieces go out as one store each, nt -- except in those two lines, which
    // the neighbouring wave writes too: those with the default policy, so that the L2 merges
    // the two waves' parts of the line before it goes to HBM (round 6: 16.2 -> 14.4 us at
    // 4096 x 4090, 15.3 -> 13.5 at 4095; profiles/r06/chunk/s3_flush_variants.jsonl).
    uint32_t span = 0;
    uintptr_t ob = 0, l_first = 0, l_last = 0;
    if constexpr (SW != 16) {
        const uint32_t cl2 = min(cw + 255u, A.chunks - 1u);
        const uint32_t rl2 = fdiv(cl2, A.L);
        const uint32_t ql2 = cl2 - rl2 * A.L.d;
        span = cw >= A.chunks ? 0u : (uint32_t)((uint64_t)rl2 * A.n + min(8u * ql2 + 8u, A.n) - e0);
        ob = (uintptr_t)A.out + 2u * e0;
        l_first = ob >> 7;
        l_last = (ob + 2u * span - 1u) >> 7;
    }
    // whole staged pieces k0 <= k < k1 (uniform bounds; piece k = elements 8k - sa .. + 7 of the span)
    auto store_pieces = [&](uint32_t k0, uint32_t k1) {
        for (uint32_t kb = k0; kb < k1; kb += 64u) {  // (uniform)
            const uint32_t k = kb + lane;
            const int x0 = (int)(8u * k) - (int)sa;
            const bool whole = k < k1 && x0 >= 0 && x0 + 8 <= (int)span;
            const u32x4 v = *reinterpret_cast<const u32x4_alias*>(stage + sbase + 16u * (k < k1 ? k : k0));
            const uint32_t off = whole ? 2u * (uint32_t)x0 : kDrop;
            const uintptr_t l = (ob + 2u * (uint32_t)x0) >> 7;
            if (l == l_first || l == l_last) __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, kAuxPiece);
            else __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, kAuxStore);
        }
    };
    // after step j (rows of >= 64 chunks): every slot below the end of the step's last chunk
    // (lane 63's) is final -- a past-n element lands only beyond its own chunk's last valid
    // one -- so the pieces wholly below it can go out now, while later steps decode, instead
    // of all after the last step (round 6)
    auto flush_step = [&](int j, uint32_t& kdone) {
        if constexpr (SW != 16) {
            const uint32_t rel63 = __builtin_amdgcn_readlane(rel[j], 63);
            const uint32_t col63 = __builtin_amdgcn_readlane(col[j], 63);
            const uint32_t e_end = col63 < A.n ? rel63 + min(8u, A.n - col63) : span;
            const uint32_t kmax = (e_end + sa) >> 3;
            store_pieces(kdone, kmax);
            kdone = kmax > kdone ? kmax : kdone;
        }
    };
    auto flush16 = [&](uint32_t kdone) {
        if constexpr (SW != 16) {
            if (cw >= A.chunks) return;  // a wave wholly past the end stages nothing and writes nothing
            store_pieces(kdone, (span + sa) >> 3);
            // The span's two end pieces when they are not whole: lane 0 the first, lane 1 the
            // last, element by element through the span's own range-checked descriptor -- the
            // elements outside the span (the neighbour's) are dropped by the range check, below
            // its start because their offsets wrap past 2^31 -- in ONE pass of 8 stores per wave
            // (round 5 made a pass per end, each with a compare per element)
            const __amdgpu_buffer_rsrc_t rsp =
                __builtin_amdgcn_make_buffer_rsrc((void*)((char*)A.out + e0 * 2u), 0, 2u * span, kRsrcFlags);
            const uint32_t klast = (span + sa - 1u) >> 3;
            const uint32_t k = lane == 0u ? 0u : klast;
            const int xe = (int)(8u * k) - (int)sa;
            if (lane < 2u && (lane == 0u || klast != 0u) && !(xe >= 0 && xe + 8 <= (int)span)) {
                const u32x4 v = *reinterpret_cast<const u32x4_alias*>(stage + sbase + 16u * k);
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(v[i >> 1] >> (16 * (i & 1))), rsp,
                                                          2u * (uint32_t)(xe + i), 0, kAuxPiece);
            }
        }
    };
    if constexpr (DT != NF4DQ_F32) {
        if (A.L.d >= 64u) {  // every wave of the launch: no workgroup barrier on this path
            // one table per block of the wave (chunk_table_build / chunk_table_decode)
            const uint32_t region = (threadIdx.x >> 6) << 11;
            chunk_table_build<DT>(ctbl, region, lane, sb);
            uint32_t kdone = 0;  // staged pieces stored so far (uniform)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t p[4];
                chunk_table_decode(ctbl, region, w[j], gsel[j], p);
                store16(j, p);
                if (j < 3 && cw < A.chunks) flush_step(j, kdone);
            }
            flush16(kdone);
            return;
        }
    }
    write_lut(lut);
    __syncthreads();
    const char* t = reinterpret_cast<const char*>(lut);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t hi4 = (w[j] >> 2) & 0x3C3C3C3Cu;
        const uint32_t lo4 = (w[j] << 2) & 0x3C3C3C3Cu;
        const float sh = __shfl(sb, (int)gsel[j], 64);
        const float sj = shared ? sh : s[j];
        float v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[2 * k] = *reinterpret_cast<const float*>(t + ((hi4 >> (8 * k)) & 0xFFu)) * sj;
            v[2 * k + 1] = *reinterpret_cast<const float*>(t + ((lo4 >> (8 * k)) & 0xFFu)) * sj;
        }
        if constexpr (DT == NF4DQ_F32) {
            const uint32_t ob = rel[j] * 4u;
            if constexpr (SW == 16) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const u32x4 o = {__float_as_uint(v[4 * h]), __float_as_uint(v[4 * h + 1]),
                                     __float_as_uint(v[4 * h + 2]), __float_as_uint(v[4 * h + 3])};
                    // (half-chunks: a store instruction writes every other 16 bytes, so the
                    // default policy, letting the L2 merge the two instructions' halves of each
                    // line: padded 4096^2 fp32 57.2 -> 18.3 us against nt, round 6 s19)
                    __builtin_amdgcn_raw_buffer_store_b128(o, ro, col[j] + 4u * h < A.n ? ob + 16u * h : kDrop, 0,
                                                           kAuxPiece);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i]), ro, col[j] + i < A.n ? ob + 4u * i : kDrop,
                                                          0, kAuxPiece);
            }
        } else {
            uint32_t p[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) p[k] = pack2<DT>(v[2 * k], v[2 * k + 1]);
            store16(j, p);
        }
    }
    if constexpr (DT != NF4DQ_F32) flush16(0u);
}

// The piece kernel (round 6): the 16-bit outputs the chunk forms above can only store
// through the LDS stage (n % 8 != 0, or the output off 16-byte alignment), for TIGHTLY
// packed rows (exactly ceil(n / 2) bytes each: every bitsandbytes weight).  It works in
// output order instead of chunk order: the output, from the 128-byte line holding its
// first element, is cut into aligned 16-byte pieces of 8 elements, and lane i owns piece
// 256 w + 64 j + i at step j of wave w.  So every whole piece is one nt 16-byte store
// straight from registers and each output line is written by one wave -- no stage, no
// line shared by two waves but the matrix's first and last.  The cost moves to the
// loads, where it is cheap: element (r, c) is nibble 2 r ceil(n / 2) + c of the packed
// stream (for even n the stream runs on across row ends, for odd n every row ends in a
// pad nibble), so a piece starts at any nibble; the lane loads the two dwords around its
// 5 bytes and forms the even and odd elements' code bytes with byte permutes and
// rotates.  A piece can hold two scale blocks (a block boundary inside the row, or the
// row's end: the next row's first block is the next block), three when a row's last block
// is shorter than a piece.  The per-block tables of 16 rounded outputs (as in the dense
// form) sit in 16 OVERLAPPING groups of 8 blocks -- group q holds blocks 4q .. 4q + 7 -- so
// the blocks of a piece lie in group tA / 4 and one v_perm per element still forms its
// table address.
struct PieceArgs {
    const uint8_t* packed;  // the packed weight aligned down to 4 bytes
    const uint8_t* a1;
    const float* a2;
    void* line;             // the output's first 128-byte line
    void* out;
    uint32_t prange;        // load range from `packed` (bytes)
    uint32_t kb;            // the weight's first byte, from `packed` (0..3)
    uint32_t sa;            // the output's first element, from `line` (0..63)
    uint32_t elems;         // m * n
    uint32_t n, half;       // columns; ceil(n / 2)
    uint32_t stride;        // packed bytes per row (>= half; > half: padded rows)
    FastDiv nf, bpr;        // n; 64-column blocks per row
    uint32_t groups;        // ceil(bpr / 4)
    FastDiv nb, n2;         // ref: moduli of the absmax / nested-absmax indices
    uint32_t rs;            // single: absmax per row
};

constexpr uint32_t kPieceTbl = 4096;  // a wave's tables: 16 groups x 8 blocks x 16 entries x 2 B

// byte 0 of x in all four bytes (one v_perm_b32; a multiply by 0x01010101 is a quarter-rate
// v_mul_lo_u32, and the constant does not fit v_mul_u32_u24's 24 bits)
__device__ __forceinline__ uint32_t bytes4(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0u); }

// One wave of a piece kernel (EP elements per 16-byte piece, 4 steps of 64 pieces): each
// step's column (of the piece's first element; < 0 before the output: wave 0's first
// pieces), its row's first block from g0, and the two packed dwords around its nibbles --
// all loads out first.  A step moves 64 EP <= 512 elements and rows are >= 512: at most one
// row end per step, so every index advances by additions.  false: the wave lies wholly
// past the end (it must return; no barrier follows in either kernel).
// RE, how a piece's elements past its row's end are found: 0 = the next nibbles (tight rows,
// even n: the stream runs on), 1 = one nibble further on (tight rows, odd n: the pad nibble),
// 2 = the next row's first bytes, loaded separately (padded rows).
template <uint32_t EP, int RE>
struct PieceWave {
    int32_t fw;              // the wave's first element (< 0: wave 0)
    uint32_t c0, g0, gl;     // column of its first element in the matrix; its first / last block
    int32_t c[4], b[4];      // per step: column, byte of nibble c from `packed`
    uint32_t gr[4], lo[4], hi[4];  // per step: the row's first block from g0; the two dwords
    uint32_t nb[4], lo2[4], hi2[4];  // RE 2, per step: the next row's first byte and its two dwords
};

template <uint32_t EP, int RE>
__device__ __forceinline__ bool piece_wave(const PieceArgs& A, uint32_t kw, uint32_t lane, PieceWave<EP, RE>& W) {
    if (EP * kw >= A.sa + A.elems) return false;
    W.fw = (int32_t)(EP * kw) - (int32_t)A.sa;
    const uint32_t fwc = W.fw < 0 ? 0u : (uint32_t)W.fw;
    const uint32_t r0 = fdiv(fwc, A.nf);
    W.c0 = fwc - r0 * A.nf.d;
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)A.packed, 0, A.prange, kRsrcFlags);
    uint32_t aj[4], an[4];
    {
        int32_t c = (W.fw < 0 ? W.fw : (int32_t)W.c0) + (int32_t)(EP * lane);
        uint32_t pb = A.kb + r0 * A.stride;  // the row's first packed byte, from `packed`
        uint32_t gb = 0u - (W.c0 >> 6);       // the row's first block, from g0
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j) c += (int32_t)(64u * EP);
            const bool wrap = c >= (int32_t)A.n;  // (additions only: no multiply per step)
            c = wrap ? c - (int32_t)A.n : c;
            pb = wrap ? pb + A.stride : pb;
            gb = wrap ? gb + A.bpr.d : gb;
            W.c[j] = c;
            W.gr[j] = gb;
            // the byte holding nibble c of the row (before the weight: negative, i.e. beyond
            // the range once unsigned -- the load returns 0)
            W.b[j] = (int32_t)pb + (c >> 1);
            aj[j] = (uint32_t)(W.b[j] & ~3);
            if constexpr (RE == 2) {
                // only a piece crossing its row's end loads the next row's first bytes
                // (past the last row: beyond the range)
                W.nb[j] = pb + A.stride;
                an[j] = c > (int32_t)(A.n - EP) ? W.nb[j] & ~3u : kDrop;
            } else {
                W.nb[j] = W.lo2[j] = W.hi2[j] = 0u;  // (unused)
                an[j] = 0u;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // the second dword's offset as its own register: folded into the instruction's offset
        // field (or the pair merged into one 8-byte load), a + 4 would be range-checked
        // unwrapped, so the weight's first dword (a = -4) would read as 0 (the first piece of
        // an output off its 128-byte line).  (8-byte loads for the waves past the first line:
        // 5-13 % slower, round 6 s14.)
        uint32_t a4 = aj[j] + 4u;
        asm("" : "+v"(a4));
        W.lo[j] = __builtin_amdgcn_raw_buffer_load_b32(rp, aj[j], 0, 0);
        W.hi[j] = __builtin_amdgcn_raw_buffer_load_b32(rp, a4, 0, 0);
        if constexpr (RE == 2) {
            uint32_t n4 = an[j] + 4u;
            asm("" : "+v"(n4));
            W.lo2[j] = __builtin_amdgcn_raw_buffer_load_b32(rp, an[j], 0, 0);
            W.hi2[j] = __builtin_amdgcn_raw_buffer_load_b32(rp, n4, 0, 0);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    W.g0 = r0 * A.bpr.d + (W.c0 >> 6);
    const uint32_t fl = min((uint32_t)(W.fw + (int32_t)(256u * EP) - 1), A.elems - 1u);
    const uint32_t rl = fdiv(fl, A.nf);
    W.gl = rl * A.bpr.d + ((fl - rl * A.nf.d) >> 6);
    return true;
}

// The scale of block min(g0 + lane, gl) (the wave's blocks are consecutive; lane i rounds
// block g0 + i's table).
template <int MODE>
__device__ __forceinline__ float piece_scale(const PieceArgs& A, uint32_t g0, uint32_t gl, uint32_t lane) {
    const uint32_t g = min(g0 + lane, gl);
    const uint32_t r = fdiv(g, A.bpr);
    const uint32_t b = g - r * A.bpr.d;
    if constexpr (MODE == kRef) {
        const float q8 = (float)A.a1[fmodu(g, A.nb)];
        return (q8 / 127.0f) * A.a2[fmodu(opaque_mul(r, A.groups) + (b >> 2), A.n2)];  // IEEE division (:45, :270)
    } else {
        return A.a2[opaque_mul(r, A.rs) + b];
    }
}

// A piece's table-address bytes: es byte i for element 2i, os byte i for element 2i + 1, each
// the element's code << SH (SH = log2 of the table entry's bytes: 1 for 16-bit, 2 for fp32)
// ORed with its block's slot in the group << (SH + 4): `slot` for the piece's first block, +1
// from each boundary on.  The boundaries (EP = elements per piece: none) are ib_in, a block
// boundary inside the row before its end, and ib_end, the row's end; with a row's last block
// at least EP long only one of them lies inside a piece (TRI false: one boundary, the smaller);
// TRI: rows whose last block is shorter than a piece, where a piece can hold three blocks.
// Nibble c of a row is the high nibble of its byte when c is even; W0 = bytes b .. b+3, W1 =
// b+1 .. b+4 of the two loaded dwords.  The elements from ib_end on come from the next row
// as RE says (PieceWave); RE 2: its first bytes are the dword pair lo2 / hi2 around byte nb.
template <int SH, int RE, bool TRI>
__device__ __forceinline__ void piece_codes(uint32_t lo, uint32_t hi, int32_t b, int32_t c, uint32_t ib_in,
                                            uint32_t ib_end, uint32_t slot, uint32_t lo2, uint32_t hi2,
                                            uint32_t nb, uint32_t& es, uint32_t& os) {
    constexpr uint32_t kCode = 0x0F0F0F0Fu << SH, kStep = 0x01010101u << (SH + 4), kEP = 16u >> SH;
    // bit SH + 4 of each byte of y(ib): the element lies at or past ib (0x80 + 2i - ib >= 0x80,
    // bytes never borrow)
    auto yE = [](uint32_t ib) { return ((0x86848280u - bytes4(ib)) >> (3 - SH)) & kStep; };
    auto yO = [](uint32_t ib) { return ((0x87858381u - bytes4(ib)) >> (3 - SH)) & kStep; };
    uint32_t sE, sO, eE, eO;  // slot increments; the bytes past the row's end
    if constexpr (TRI) {
        eE = yE(ib_end);
        eO = yO(ib_end);
        sE = eE + yE(ib_in);
        sO = eO + yO(ib_in);
    } else {
        sE = yE(min(ib_in, ib_end));
        sO = yO(min(ib_in, ib_end));
        eE = ib_end < kEP ? sE : 0u;
        eO = ib_end < kEP ? sO : 0u;
    }
    const uint32_t sel = bytes4((uint32_t)b & 3u) + 0x03020100u;
    const uint32_t w0 = __builtin_amdgcn_perm(hi, lo, sel);
    const uint32_t w1 = __builtin_amdgcn_perm(hi, lo, sel + 0x01010101u);
    const uint32_t h0 = __builtin_amdgcn_alignbit(w0, w0, 4u - SH);   // high nibbles << SH
    const uint32_t l0 = __builtin_amdgcn_alignbit(w0, w0, 32u - SH);  // low nibbles << SH
    const uint32_t h1 = __builtin_amdgcn_alignbit(w1, w1, 4u - SH);
    const bool odd = (c & 1) != 0;
    uint32_t E = odd ? l0 : h0, O = odd ? h1 : l0;
    if constexpr (RE != 0) {
        uint32_t E2, O2;  // the codes the elements past the row's end take, in place
        if constexpr (RE == 1) {  // one nibble further on
            const uint32_t l1 = __builtin_amdgcn_alignbit(w1, w1, 32u - SH);
            E2 = O;
            O2 = odd ? l1 : h1;
        } else {  // element i >= e = ib_end is column i - e of the next row (an even start)
            const uint32_t wn = __builtin_amdgcn_perm(hi2, lo2, bytes4(nb & 3u) + 0x03020100u);
            const uint32_t hn = __builtin_amdgcn_alignbit(wn, wn, 4u - SH);
            const uint32_t ln = __builtin_amdgcn_alignbit(wn, wn, 32u - SH);
            const uint32_t e = ib_end, eodd = e & 1u;
            E2 = (eodd ? ln : hn) << ((8u * ((e + 1u) >> 1)) & 31u);  // (e = EP: masked out below)
            O2 = (eodd ? hn : ln) << ((8u * (e >> 1)) & 31u);
        }
        const uint32_t kE = eE - (eE >> 4);  // the code bits of the bytes past the row's end
        const uint32_t kO = eO - (eO >> 4);
        E = (E2 & kE) | (E & ~kE);
        O = (O2 & kO) | (O & ~kO);
    }
    const uint32_t rep = bytes4(slot << (SH + 4));
    es = (E & kCode) | (rep + sE);
    os = (O & kCode) | (rep + sO);
}

template <int DT, int MODE, int RE, bool TRI>
__global__ __launch_bounds__(kWg) void nf4_piece_kernel(const PieceArgs A) {
    __shared__ __attribute__((aligned(256))) char ptbl[4 * kPieceTbl];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t kw = __builtin_amdgcn_readfirstlane((blockIdx.x * 4u + (threadIdx.x >> 6)) * 256u);
    PieceWave<8, RE> W;
    if (!piece_wave<8, RE>(A, kw, lane, W)) return;  // (uniform)
    const float sb = piece_scale<MODE>(A, W.g0, W.gl, lane);
    const uint32_t region = (threadIdx.x >> 6) * kPieceTbl;
    {
        uint32_t e[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            e[k] = pack2<DT>(__uint_as_float(kNf4Bits[2 * k]) * sb, __uint_as_float(kNf4Bits[2 * k + 1]) * sb);
        // block i: slot i % 4 of group i / 4, and slot i % 4 + 4 of group i / 4 - 1
        u32x4_alias* d0 = reinterpret_cast<u32x4_alias*>(ptbl + region + ((lane >> 2) << 8) + ((lane & 3u) << 5));
        d0[0] = u32x4{e[0], e[1], e[2], e[3]};
        d0[1] = u32x4{e[4], e[5], e[6], e[7]};
        if (lane >= 4u) {
            u32x4_alias* d1 = reinterpret_cast<u32x4_alias*>(ptbl + region + ((lane >> 2) << 8) - 256u + 128u +
                                                            ((lane & 3u) << 5));
            d1[0] = u32x4{e[0], e[1], e[2], e[3]};
            d1[1] = u32x4{e[4], e[5], e[6], e[7]};
        }
    }
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(A.line, 0, 2u * (A.sa + A.elems), kRsrcFlags);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // (c < 0: wave 0's first pieces, whose elements are block 0's or dropped)
        const uint32_t cu = (uint32_t)max(W.c[j], 0);
        // the piece's first block (from g0) and the elements where the next blocks start (8:
        // none): a block boundary inside the row, the row's end (see piece_codes)
        const uint32_t tA = min(W.gr[j] + (cu >> 6), 59u);  // (59: lanes past the end)
        const uint32_t to_blk = 64u - (cu & 63u), to_end = A.n - cu;
        const uint32_t ib_in = to_blk < to_end ? min(to_blk, 8u) : 8u, ib_end = min(to_end, 8u);
        uint32_t es, os;
        piece_codes<1, RE, TRI>(W.lo[j], W.hi[j], W.b[j], W.c[j], ib_in, ib_end, tA & 3u, W.lo2[j], W.hi2[j],
                                W.nb[j], es, os);
        const uint32_t base = region + ((tA >> 2) << 8);
        uint32_t p[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t ve = *reinterpret_cast<const u16_alias*>(ptbl + __builtin_amdgcn_perm(es, base, 0x03020104u + b));
            const uint32_t vo = *reinterpret_cast<const u16_alias*>(ptbl + __builtin_amdgcn_perm(os, base, 0x03020104u + b));
            p[b] = __builtin_amdgcn_perm(vo, ve, 0x05040100u);  // (one v_perm; the compiler made shift + or_sdwa)
        }
        const uint32_t k = kw + 64u * (uint32_t)j + lane;
        const int32_t f = W.fw + 8 * (64 * j + (int32_t)lane);
        const bool whole = f >= 0 && (uint32_t)f + 8u <= A.elems;
        const u32x4 o = {p[0], p[1], p[2], p[3]};
        __builtin_amdgcn_raw_buffer_store_b128(o, ro, whole ? 16u * k : kDrop, 0, kAuxStore);
        if (!whole && f < (int32_t)A.elems && f + 8 > 0) {
            // the matrix's first or last piece, partly outside the output: element by element
            // through the output's own range (offsets before it wrap past 2^31: dropped)
            const __amdgpu_buffer_rsrc_t rsp =
                __builtin_amdgcn_make_buffer_rsrc(A.out, 0, 2u * A.elems, kRsrcFlags);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t oe = 2u * (uint32_t)(f + i);
                asm("" : "+v"(oe));  // (each offset its own register: see piece_wave)
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(p[i >> 1] >> (16 * (i & 1))), rsp, oe, 0,
                                                      kAuxPiece);
            }
        }
    }
}

// The piece kernel's fp32 form (quant_state.dtype = torch.float32): a piece is 4 elements,
// so a wave's step covers 256 elements and its store 1 KiB.  Every tight fp32 shape the flat
// kernel does not take comes here: the chunk kernel's fp32 stores (two 16-byte halves of a
// 32-byte chunk per lane, or element stores) write 128-byte lines in pieces from several
// instructions, 47-58 us for 4096 x 4080..4096 against 13.3 for the flat kernel at 4096^2
// (profiles/r06/chunk/s17_f32_forms.jsonl).  The per-block tables hold the 16 fp32 products
// (64 bytes, no rounding); group q holds blocks 2q .. 2q + 3, so a piece's two blocks share a
// 256-byte group and an element's table address is one v_perm of its code byte (code x 4 in
// bits 2..5, slot x 64 in bits 6..7).
constexpr uint32_t kPiece32Tbl = 12 * 256;  // a wave's tables: blocks 0 .. 23 (a wave touches <= 20)

template <int MODE, int RE, bool TRI>
__global__ __launch_bounds__(kWg) void nf4_piece32_kernel(const PieceArgs A) {
    __shared__ __attribute__((aligned(256))) char ptbl[4 * kPiece32Tbl];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t kw = __builtin_amdgcn_readfirstlane((blockIdx.x * 4u + (threadIdx.x >> 6)) * 256u);
    PieceWave<4, RE> W;
    if (!piece_wave<4, RE>(A, kw, lane, W)) return;  // (uniform)
    const float sb = piece_scale<MODE>(A, W.g0, W.gl, lane);
    const uint32_t region = (threadIdx.x >> 6) * kPiece32Tbl;
    if (lane < 24u) {
        // block i: slot i % 2 of group i / 2, and slot i % 2 + 2 of group i / 2 - 1
        u32x4 e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            e[k] = u32x4{__float_as_uint(__uint_as_float(kNf4Bits[4 * k]) * sb),
                         __float_as_uint(__uint_as_float(kNf4Bits[4 * k + 1]) * sb),
                         __float_as_uint(__uint_as_float(kNf4Bits[4 * k + 2]) * sb),
                         __float_as_uint(__uint_as_float(kNf4Bits[4 * k + 3]) * sb)};  // (:97-98)
        u32x4_alias* d0 = reinterpret_cast<u32x4_alias*>(ptbl + region + ((lane >> 1) << 8) + ((lane & 1u) << 6));
#pragma unroll
        for (int k = 0; k < 4; ++k) d0[k] = e[k];
        if (lane >= 2u) {
            u32x4_alias* d1 = reinterpret_cast<u32x4_alias*>(ptbl + region + ((lane >> 1) << 8) - 256u + 128u +
                                                            ((lane & 1u) << 6));
#pragma unroll
            for (int k = 0; k < 4; ++k) d1[k] = e[k];
        }
    }
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(A.line, 0, 4u * (A.sa + A.elems), kRsrcFlags);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t cu = (uint32_t)max(W.c[j], 0);
        const uint32_t tA = min(W.gr[j] + (cu >> 6), 21u);  // (21: lanes past the end)
        const uint32_t to_blk = 64u - (cu & 63u), to_end = A.n - cu;
        const uint32_t ib_in = to_blk < to_end ? min(to_blk, 4u) : 4u, ib_end = min(to_end, 4u);
        uint32_t es, os;
        piece_codes<2, RE, TRI>(W.lo[j], W.hi[j], W.b[j], W.c[j], ib_in, ib_end, tA & 1u, W.lo2[j], W.hi2[j],
                                W.nb[j], es, os);
        const uint32_t base = region + ((tA >> 1) << 8);
        uint32_t p[4];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            p[2 * b] = *reinterpret_cast<const uint32_t*>(ptbl + __builtin_amdgcn_perm(es, base, 0x03020104u + b));
            p[2 * b + 1] = *reinterpret_cast<const uint32_t*>(ptbl + __builtin_amdgcn_perm(os, base, 0x03020104u + b));
        }
        const uint32_t k = kw + 64u * (uint32_t)j + lane;
        const int32_t f = W.fw + 4 * (64 * j + (int32_t)lane);
        const bool whole = f >= 0 && (uint32_t)f + 4u <= A.elems;
        const u32x4 o = {p[0], p[1], p[2], p[3]};
        __builtin_amdgcn_raw_buffer_store_b128(o, ro, whole ? 16u * k : kDrop, 0, kAuxStore);
        if (!whole && f < (int32_t)A.elems && f + 4 > 0) {
            const __amdgpu_buffer_rsrc_t rsp =
                __builtin_amdgcn_make_buffer_rsrc(A.out, 0, 4u * A.elems, kRsrcFlags);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t oe = 4u * (uint32_t)(f + i);
                asm("" : "+v"(oe));
                __builtin_amdgcn_raw_buffer_store_b32(p[i], rsp, oe, 0, kAuxPiece);
            }
        }
    }
}

// Any length, bitsandbytes semantics: one thread per packed byte.
struct BnbBytesArgs {
    const uint8_t* packed;
    const uint8_t* a1;
    const float* code2;
    const float* a2;
    void* out;
    float offset;
    int64_t numel;
    int32_t blk_shift_elems, blk2_shift;
    int32_t single;
};

template <int DT>
__global__ __launch_bounds__(kWg) void nf4_bnb_bytes_kernel(const BnbBytesArgs A) {
    __shared__ __attribute__((aligned(16))) float lut[16];
    write_lut(lut);
    __syncthreads();
    const int64_t nbytes = (A.numel + 1) / 2;
    for (int64_t i = (int64_t)blockIdx.x * kWg + threadIdx.x; i < nbytes; i += (int64_t)gridDim.x * kWg) {
        const int64_t e = 2 * i;
        const int64_t blk = e >> A.blk_shift_elems;
        const float s = A.single ? A.a2[blk] : A.code2[A.a1[blk]] * A.a2[blk >> A.blk2_shift] + A.offset;
        const uint32_t byte = A.packed[i];
        store1<DT>(A.out, e, lut[byte >> 4] * s);
        if (e + 1 < A.numel) store1<DT>(A.out, e + 1, lut[byte & 15u] * s);
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
inline int hip_rc(hipError_t e) { return e == hipSuccess ? NF4DQ_OK : NF4DQ_ERR_HIP_BASE + (int)e; }

inline bool valid_dtype(int32_t d) { return d == NF4DQ_F16 || d == NF4DQ_BF16 || d == NF4DQ_F32; }

inline bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

inline int ilog2(uint64_t v) {
    int s = 0;
    while ((uint64_t(1) << s) < v) ++s;
    return s;
}

constexpr nf4_launch_cfg kDefaultCfg = {4, 0, 1, 0};  // measured best at 4096^2 (tools/tune.py)

#if NF4_FLAT_STAMPS
unsigned long long* g_stamps = nullptr;  // diagnostic build: [wave][4] u64
#endif

int cu_count() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 256;
    return cus;
}

template <int DT, int MODE, int MAXB>
void launch_one(const Batch<MAXB>& b, uint64_t blocks, hipStream_t st) {
    hipLaunchKernelGGL((nf4_flat_kernel<DT, MODE, MAXB>), dim3((unsigned)blocks), dim3(kFlatWg), 0, st, b);
}

// Launch one flat batch.  Tile offsets are (re)computed here for the tile size of
// the dtype; callers only fill the per-matrix descriptors.  cfg: grid cap
// (blocks_per_cu), validated by the caller.
template <int MAXB>
int launch_flat_batch(const Batch<MAXB>& bt, int dtype, int mode, const nf4_launch_cfg& cfg, hipStream_t st) {
    if (bt.count == 0) return NF4DQ_OK;
    const uint32_t tb = 64u * (dtype == NF4DQ_F32 ? 2u : 4u) * kU;
    Batch<MAXB> b = bt;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < b.count; ++i) {
        b.d[i].tile_begin = acc;
        acc += (b.d[i].nbytes + tb - 1u) / tb;
    }
    b.total_tiles = acc;
    if (acc == 0) return NF4DQ_OK;
    uint64_t blocks = (acc + kFlatWaves - 1) / kFlatWaves;
    if (cfg.blocks_per_cu > 0) {
        const uint64_t cap = (uint64_t)cfg.blocks_per_cu * (uint64_t)cu_count();
        if (blocks > cap) blocks = cap;
    }
#if NF4_FLAT_STAMPS
    b.stamps = g_stamps;
#endif
#define NF4_D(DT_)                                                              \
    do {                                                                        \
        switch (mode) {                                                         \
            case kRef: launch_one<DT_, kRef, MAXB>(b, blocks, st); break;       \
            case kSingle: launch_one<DT_, kSingle, MAXB>(b, blocks, st); break; \
            case kBnb: launch_one<DT_, kBnb, MAXB>(b, blocks, st); break;       \
            default: launch_one<DT_, kBnbSingle, MAXB>(b, blocks, st); break;   \
        }                                                                       \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_D(NF4DQ_BF16);
    else if (dtype == NF4DQ_F16) NF4_D(NF4DQ_F16);
    else NF4_D(NF4DQ_F32);
#undef NF4_D
    return hip_rc(hipGetLastError());
}

inline unsigned rows_grid(int64_t work) {
    int64_t b = (work + kWg - 1) / kWg;
    if (b > 65536) b = 65536;  // grid-stride beyond this
    if (b < 1) b = 1;
    return (unsigned)b;
}

// Validation shared by the reference-semantics entry points (mirrors what the
// reference's .view(m, -1) and slicing accept, kernel_optimized.py:229, :288-312).
int check_common(const uint8_t* packed, int64_t packed_len, const void* out, int32_t dtype, int64_t m, int64_t n) {
    if (!valid_dtype(dtype)) return NF4DQ_ERR_ARG;
    if (m < 0 || n < 0 || packed_len < 0) return NF4DQ_ERR_ARG;
    if (m == 0 || n == 0) return NF4DQ_OK;
    if (!packed || !out) return NF4DQ_ERR_ARG;
    if (packed_len % m) return NF4DQ_ERR_SHAPE;
    if (packed_len / m < (n + 1) / 2) return NF4DQ_ERR_SHAPE;
    return NF4DQ_OK;
}

// Fill a flat-path descriptor for reference / single semantics, or return false
// when the matrix needs the rows kernel.
// Buffer descriptors address < 4 GiB: a flat piece holds < 2^29 packed bytes
// (2 GiB of 16-bit / 4 GiB of fp32 output).  Bigger matrices (a 70B model's
// 128256 x 8192 lm_head) go as several row-aligned pieces of one launch, each
// carrying its first scale block (Desc::blk_base); block indices stay < 2^31.
constexpr int64_t kPieceBytes = int64_t(1) << 29;
constexpr int64_t kMaxFlatBlocks = int64_t(1) << 31;

bool flat_eligible(const uint8_t* packed, int64_t packed_len, const void* out, int64_t m, int64_t n) {
    return n % 64 == 0 && packed_len == m * (n / 2) && n / 2 < kPieceBytes && packed_len / 32 < kMaxFlatBlocks &&
           aligned(packed, 4) && aligned(out, 16);
}

// Rows per piece of a flat-eligible matrix with n columns.
inline int64_t piece_rows(int64_t n) { return (kPieceBytes - 1) / (n / 2); }

// Append the row pieces of one flat-eligible matrix (descriptor `proto` covers
// the whole matrix) to batch `b`, launching whenever it fills.
template <int MAXB>
int append_pieces(Batch<MAXB>& b, const Desc& proto, int64_t m, int64_t n, int32_t dtype, int mode,
                  hipStream_t st) {
    const int64_t rows = piece_rows(n);
    const int64_t ob = dtype == NF4DQ_F32 ? 4 * n : 2 * n;
    for (int64_t r0 = 0; r0 < m; r0 += rows) {
        const int64_t r1 = r0 + rows < m ? r0 + rows : m;
        Desc d = proto;
        d.packed = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(proto.packed) + r0 * (n / 2));
        d.out = reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(proto.out) + r0 * ob);
        d.nbytes = (uint32_t)((r1 - r0) * (n / 2));
        d.blk_base = (uint32_t)(r0 * (n / 64));
        d.tile_begin = b.total_tiles;
        b.d[b.count++] = d;
        b.total_tiles += (d.nbytes + 1023u) / 1024u;
        if (b.count == (uint32_t)MAXB || b.total_tiles > (1u << 30)) {
            const int rc = launch_flat_batch(b, dtype, mode, kDefaultCfg, st);
            if (rc) return rc;
            b.count = 0;
            b.total_tiles = 0;
        }
    }
    return NF4DQ_OK;
}

// One flat-eligible matrix: a single-descriptor launch, or pieces.
int launch_flat_matrix(const Desc& proto, int64_t m, int64_t n, int32_t dtype, int mode, const nf4_launch_cfg& cfg,
                       hipStream_t st) {
    const int64_t packed_len = m * (n / 2);
    if (packed_len < kPieceBytes) {
        Batch<1> b{};
        b.d[0] = proto;
        b.d[0].nbytes = (uint32_t)packed_len;
        b.count = 1;
        b.total_tiles = (uint32_t)((packed_len + 1023) / 1024);
        return launch_flat_batch(b, dtype, mode, cfg, st);
    }
    Batch<NF4DQ_BATCH_MAX> b{};
    const int rc = append_pieces(b, proto, m, n, dtype, mode, st);
    if (rc || b.count == 0) return rc;
    return launch_flat_batch(b, dtype, mode, kDefaultCfg, st);
}

Desc ref_desc(const uint8_t* packed, int64_t packed_len, const uint8_t* a1, int64_t nb, const float* a2,
              int64_t n2, void* out, int64_t n) {
    Desc d{};
    d.packed = reinterpret_cast<const uint32_t*>(packed);
    d.a1 = a1;
    d.a2 = a2;
    d.out = reinterpret_cast<u32x4*>(out);
    d.nbytes = packed_len < kPieceBytes ? (uint32_t)packed_len : 0u;  // pieces set their own
    const int64_t bpr = (n + 63) / 64;
    d.groups = (uint32_t)((bpr + 3) / 4);
    // moduli above 2^31 never wrap for indices < 2^31: clamp keeps FastDiv valid
    d.nb = make_fastdiv((uint32_t)(nb > (int64_t(1) << 31) ? (int64_t(1) << 31) : nb));
    d.n2 = make_fastdiv((uint32_t)(n2 > (int64_t(1) << 31) ? (int64_t(1) << 31) : n2));
    d.bpr = make_fastdiv((uint32_t)bpr);
    d.blk_shift = 5;  // 64 elements = 32 packed bytes
    return d;
}

// Fill the chunk kernel's shape fields, or return false when the matrix is past its
// limits: every index it forms is 32-bit (chunks, blocks, scale indices, offsets within
// the rows one wave's 256 chunks touch) and its stores need element-aligned output.
bool chunk_args(ChunkArgs& A, const uint8_t* packed, int64_t packed_len, void* out, int32_t dtype, int64_t m,
                int64_t n) {
    const int64_t stride = packed_len / m;
    const int64_t L = ((n + 1) / 2 + 3) / 4;
    const int64_t bpr = (n + 63) / 64;
    const int64_t ob = dtype == NF4DQ_F32 ? 4 : 2;
    const int64_t span = 256 / L + 2;  // rows one wave touches, at most
    const int64_t lim = int64_t(1) << 31;
    if (m * L >= lim - 1024 || m * bpr >= lim || n >= (int64_t(1) << 28) || span * stride >= lim ||
        span * n * ob >= lim || !aligned(out, (uintptr_t)ob))
        return false;
    A.packed = packed;
    A.out = out;
    A.packed_len = (uint64_t)packed_len;
    A.out_elems = (uint64_t)(m * n);
    A.stride = (uint32_t)stride;
    A.n = (uint32_t)n;
    A.chunks = (uint32_t)(m * L);
    A.L = make_fastdiv((uint32_t)L);
    A.bpr = make_fastdiv((uint32_t)bpr);
    A.groups = (uint32_t)((bpr + 3) / 4);
    return true;
}

template <int DT, int MODE, int LW>
void launch_chunks_lw(const ChunkArgs& A, int sw, unsigned g, hipStream_t st) {
    if (sw == 16) hipLaunchKernelGGL((nf4_chunk_kernel<DT, MODE, LW, 16>), dim3(g), dim3(kWg), 0, st, A);
    else hipLaunchKernelGGL((nf4_chunk_kernel<DT, MODE, LW, 4>), dim3(g), dim3(kWg), 0, st, A);
}

// The dense form's shapes (checked first).
bool dense_eligible(const ChunkArgs& A, int32_t dtype) {
    return dtype != NF4DQ_F32 && A.L.d >= 64u && A.stride == 4u * A.L.d && A.n % 8u == 0 && aligned(A.packed, 4) &&
           aligned(A.out, 16) && A.chunks < (1u << 27);
}

// The piece kernels' shapes: rows of >= 512 elements (a step then crosses at most one row end)
// the dense form does not take (16-bit output: n % 8 != 0, padded rows, the output off
// 16-byte alignment or the packed weight off 4-byte alignment; fp32: every such shape), and
// offsets below 2^31.
bool piece_eligible(const ChunkArgs& A, int32_t dtype) {
    const uint64_t half = (A.n + 1u) / 2u;
    const uint64_t rows = A.out_elems / A.n;
    const uint64_t ob = dtype == NF4DQ_F32 ? 4u : 2u;
    // (padded 16-bit rows the chunk kernel stores whole, n % 8 == 0 and an aligned output,
    // stay there: the same time, two loads fewer per piece; profiles/r06/chunk/s22)
    if (A.stride != half && dtype != NF4DQ_F32 && A.n % 8u == 0 && aligned(A.out, 16)) return false;
    return A.stride >= half && A.packed_len == rows * A.stride && A.n >= 512u &&
           ob * (A.out_elems + 64u) < (uint64_t(1) << 31) && A.packed_len + 8u < (uint64_t(1) << 31);
}

template <int MODE, int DT, int RE, bool TRI>
void launch_pieces_k(const PieceArgs& P, unsigned g, hipStream_t st) {
    if constexpr (DT == NF4DQ_F32) hipLaunchKernelGGL((nf4_piece32_kernel<MODE, RE, TRI>), dim3(g), dim3(kWg), 0, st, P);
    else hipLaunchKernelGGL((nf4_piece_kernel<DT, MODE, RE, TRI>), dim3(g), dim3(kWg), 0, st, P);
}

template <int MODE, int DT, int RE>
void launch_pieces_re(const PieceArgs& P, unsigned g, hipStream_t st) {
    // TRI: the last block of a row is shorter than a piece (a piece can hold three blocks)
    const uint32_t tail = P.n % 64u;
    if (tail != 0u && tail < (DT == NF4DQ_F32 ? 4u : 8u)) launch_pieces_k<MODE, DT, RE, true>(P, g, st);
    else launch_pieces_k<MODE, DT, RE, false>(P, g, st);
}

template <int MODE, int DT>
void launch_pieces_dt(const PieceArgs& P, unsigned g, hipStream_t st) {
    if (P.stride != P.half) launch_pieces_re<MODE, DT, 2>(P, g, st);  // padded rows
    else if (P.n & 1u) launch_pieces_re<MODE, DT, 1>(P, g, st);
    else launch_pieces_re<MODE, DT, 0>(P, g, st);
}

template <int MODE>
int launch_pieces(const ChunkArgs& A, int32_t dtype, hipStream_t st) {
    PieceArgs P{};
    const uint32_t ob = dtype == NF4DQ_F32 ? 4u : 2u, per = 16u / ob;  // output bytes, elements per piece
    const uintptr_t pw = (uintptr_t)A.packed, ow = (uintptr_t)A.out;
    P.packed = reinterpret_cast<const uint8_t*>(pw & ~uintptr_t(3));
    P.kb = (uint32_t)(pw & 3u);
    P.prange = (uint32_t)((P.kb + A.packed_len + 3u) & ~uint64_t(3));
    P.a1 = A.a1;
    P.a2 = A.a2;
    P.out = A.out;
    P.line = reinterpret_cast<void*>(ow & ~uintptr_t(127));
    P.sa = (uint32_t)((ow & 127u) / ob);
    P.elems = (uint32_t)A.out_elems;
    P.n = A.n;
    P.half = (A.n + 1u) / 2u;
    P.stride = A.stride;
    P.nf = make_fastdiv(A.n);
    P.bpr = A.bpr;
    P.groups = A.groups;
    P.nb = A.nb;
    P.n2 = A.n2;
    P.rs = A.rs;
    const uint32_t pieces = (P.sa + P.elems + per - 1u) / per;
    const unsigned g = (pieces + 1023u) / 1024u;  // 4 waves x 256 pieces
    if (dtype == NF4DQ_BF16) launch_pieces_dt<MODE, NF4DQ_BF16>(P, g, st);
    else if (dtype == NF4DQ_F16) launch_pieces_dt<MODE, NF4DQ_F16>(P, g, st);
    else launch_pieces_dt<MODE, NF4DQ_F32>(P, g, st);
    return hip_rc(hipGetLastError());
}

template <int MODE>
int launch_chunks(const ChunkArgs& A, int32_t dtype, hipStream_t st) {
    const unsigned g = (unsigned)((A.chunks + 1023u) / 1024u);  // 4 waves x 256 chunks
    if (!dense_eligible(A, dtype) && piece_eligible(A, dtype)) return launch_pieces<MODE>(A, dtype, st);
    if (dense_eligible(A, dtype)) {
        if (dtype == NF4DQ_BF16) hipLaunchKernelGGL((nf4_chunk_dense_kernel<NF4DQ_BF16, MODE>), dim3(g), dim3(kWg), 0, st, A);
        else hipLaunchKernelGGL((nf4_chunk_dense_kernel<NF4DQ_F16, MODE>), dim3(g), dim3(kWg), 0, st, A);
        return hip_rc(hipGetLastError());
    }
    const int lw = aligned(A.packed, 4) && A.stride % 4 == 0 ? 4 : 1;
    int sw;
    if (dtype == NF4DQ_F32) sw = A.n % 4 == 0 && aligned(A.out, 16) ? 16 : 4;
    else sw = A.n % 8 == 0 && aligned(A.out, 16) ? 16 : 4;  // (4: staged through LDS)
#define NF4_C(DT_)                                                                 \
    do {                                                                           \
        if (lw == 4) launch_chunks_lw<DT_, MODE, 4>(A, sw, g, st);                 \
        else launch_chunks_lw<DT_, MODE, 1>(A, sw, g, st);                         \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_C(NF4DQ_BF16);
    else if (dtype == NF4DQ_F16) NF4_C(NF4DQ_F16);
    else NF4_C(NF4DQ_F32);
#undef NF4_C
    return hip_rc(hipGetLastError());
}

inline FastDiv clamped_fastdiv(int64_t d) {  // moduli above 2^31 never wrap for indices < 2^31
    return make_fastdiv((uint32_t)(d > (int64_t(1) << 31) ? (int64_t(1) << 31) : d));
}

int ref_impl(const uint8_t* packed, int64_t packed_len, const uint8_t* a1, int64_t nb, const float* a2, int64_t n2,
             void* out, int32_t dtype, int64_t m, int64_t n, const nf4_launch_cfg& cfg, hipStream_t st) {
    int rc = check_common(packed, packed_len, out, dtype, m, n);
    if (rc || m == 0 || n == 0) return rc;
    if (!a1 || !a2 || nb <= 0 || n2 <= 0) return NF4DQ_ERR_ARG;
    const bool rows_only = cfg.flags & NF4DQ_CFG_ROWS, chunks = cfg.flags & NF4DQ_CFG_CHUNKS;
    if (!rows_only && !chunks && flat_eligible(packed, packed_len, out, m, n))
        return launch_flat_matrix(ref_desc(packed, packed_len, a1, nb, a2, n2, out, n), m, n, dtype, kRef, cfg, st);
    ChunkArgs C{};
    if (!rows_only && chunk_args(C, packed, packed_len, out, dtype, m, n)) {
        C.a1 = a1;
        C.a2 = a2;
        C.nb = clamped_fastdiv(nb);
        C.n2 = clamped_fastdiv(n2);
        return launch_chunks<kRef>(C, dtype, st);
    }
    RowsArgs A{};
    A.packed = packed;
    A.a1 = a1;
    A.a2 = a2;
    A.out = out;
    A.m = m;
    A.n = n;
    A.stride = packed_len / m;
    A.cols_b = (n + 1) / 2;
    A.nb = nb;
    A.n2 = n2;
    A.bpr = (n + 63) / 64;
    A.groups = (A.bpr + 3) / 4;
    const unsigned g = rows_grid(m * A.cols_b);
    if (dtype == NF4DQ_BF16) hipLaunchKernelGGL((nf4_rows_kernel<NF4DQ_BF16, kRef>), dim3(g), dim3(kWg), 0, st, A);
    else if (dtype == NF4DQ_F16) hipLaunchKernelGGL((nf4_rows_kernel<NF4DQ_F16, kRef>), dim3(g), dim3(kWg), 0, st, A);
    else hipLaunchKernelGGL((nf4_rows_kernel<NF4DQ_F32, kRef>), dim3(g), dim3(kWg), 0, st, A);
    return hip_rc(hipGetLastError());
}

}  // namespace

extern "C" {

int nf4_dequant_ref(const uint8_t* packed, int64_t packed_len, const uint8_t* absmax_q, int64_t nb,
                    const float* absmax2, int64_t n2, void* out, int32_t out_dtype, int64_t m, int64_t n,
                    void* hip_stream) {
    return ref_impl(packed, packed_len, absmax_q, nb, absmax2, n2, out, out_dtype, m, n, kDefaultCfg,
                    reinterpret_cast<hipStream_t>(hip_stream));
}

int nf4_dequant_ref_cfg(const uint8_t* packed, int64_t packed_len, const uint8_t* absmax_q, int64_t nb,
                        const float* absmax2, int64_t n2, void* out, int32_t out_dtype, int64_t m, int64_t n,
                        const nf4_launch_cfg* cfg, void* hip_stream) {
    nf4_launch_cfg c = cfg ? *cfg : kDefaultCfg;
    if (c.tile_dwords != 4 || c.nontemporal != 1 || c.blocks_per_cu < 0) return NF4DQ_ERR_ARG;
    if (c.flags & ~(NF4DQ_CFG_ROWS | NF4DQ_CFG_CHUNKS)) return NF4DQ_ERR_ARG;
    if ((c.flags & NF4DQ_CFG_ROWS) && (c.flags & NF4DQ_CFG_CHUNKS)) return NF4DQ_ERR_ARG;
    return ref_impl(packed, packed_len, absmax_q, nb, absmax2, n2, out, out_dtype, m, n, c,
                    reinterpret_cast<hipStream_t>(hip_stream));
}

int nf4_dequant_single(const uint8_t* packed, int64_t packed_len, const float* absmax, int64_t absmax_len,
                       void* out, int32_t out_dtype, int64_t m, int64_t n, void* hip_stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    int rc = check_common(packed, packed_len, out, out_dtype, m, n);
    if (rc || m == 0 || n == 0) return rc;
    if (!absmax || absmax_len < 0) return NF4DQ_ERR_ARG;
    const int64_t bpr = (n + 63) / 64;
    if (absmax_len % m || absmax_len / m < bpr) return NF4DQ_ERR_SHAPE;
    const int64_t rs = absmax_len / m;
    if (flat_eligible(packed, packed_len, out, m, n) && absmax_len < (int64_t(1) << 31)) {
        Desc d = ref_desc(packed, packed_len, nullptr, 1, absmax, 1, out, n);
        d.n2 = make_fastdiv((uint32_t)rs);
        return launch_flat_matrix(d, m, n, out_dtype, kSingle, kDefaultCfg, st);
    }
    ChunkArgs C{};
    if (m * rs < (int64_t(1) << 31) && chunk_args(C, packed, packed_len, out, out_dtype, m, n)) {
        C.a2 = absmax;
        C.rs = (uint32_t)rs;
        return launch_chunks<kSingle>(C, out_dtype, st);
    }
    RowsArgs A{};
    A.packed = packed;
    A.a2 = absmax;
    A.out = out;
    A.m = m;
    A.n = n;
    A.stride = packed_len / m;
    A.cols_b = (n + 1) / 2;
    A.bpr = bpr;
    A.rs = rs;
    const unsigned g = rows_grid(m * A.cols_b);
    if (out_dtype == NF4DQ_BF16) hipLaunchKernelGGL((nf4_rows_kernel<NF4DQ_BF16, kSingle>), dim3(g), dim3(kWg), 0, st, A);
    else if (out_dtype == NF4DQ_F16) hipLaunchKernelGGL((nf4_rows_kernel<NF4DQ_F16, kSingle>), dim3(g), dim3(kWg), 0, st, A);
    else hipLaunchKernelGGL((nf4_rows_kernel<NF4DQ_F32, kSingle>), dim3(g), dim3(kWg), 0, st, A);
    return hip_rc(hipGetLastError());
}

int nf4_dequant_ref_batched(const nf4_matrix_desc* descs, int32_t count, int32_t out_dtype, void* hip_stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    if (count < 0 || (count > 0 && !descs)) return NF4DQ_ERR_ARG;
    if (!valid_dtype(out_dtype)) return NF4DQ_ERR_ARG;
    // Validate everything before launching anything.
    for (int32_t i = 0; i < count; ++i) {
        const nf4_matrix_desc& d = descs[i];
        int rc = check_common(d.packed, d.packed_len, d.out, out_dtype, d.m, d.n);
        if (rc) return rc;
        if (d.m == 0 || d.n == 0) continue;
        if (!d.absmax_q || !d.absmax2 || d.nb <= 0 || d.n2 <= 0) return NF4DQ_ERR_ARG;
    }
    Batch<NF4DQ_BATCH_MAX> b{};
    b.count = 0;
    b.total_tiles = 0;
    for (int32_t i = 0; i < count; ++i) {
        const nf4_matrix_desc& d = descs[i];
        if (d.m == 0 || d.n == 0) continue;
        if (!flat_eligible(d.packed, d.packed_len, d.out, d.m, d.n)) {
            int rc = ref_impl(d.packed, d.packed_len, d.absmax_q, d.nb, d.absmax2, d.n2, d.out, out_dtype, d.m, d.n,
                              kDefaultCfg, st);
            if (rc) return rc;
            continue;
        }
        const int rc = append_pieces(b, ref_desc(d.packed, d.packed_len, d.absmax_q, d.nb, d.absmax2, d.n2, d.out,
                                                 d.n), d.m, d.n, out_dtype, kRef, st);
        if (rc) return rc;
    }
    if (b.count) return launch_flat_batch(b, out_dtype, kRef, kDefaultCfg, st);
    return NF4DQ_OK;
}

static int bnb_common(const uint8_t* packed, const uint8_t* a1, int64_t nb, const float* code2, const float* a2,
                      int64_t n2, float offset, void* out, int32_t dtype, int64_t numel, int32_t blocksize,
                      int32_t blocksize2, bool single, hipStream_t st) {
    if (!valid_dtype(dtype)) return NF4DQ_ERR_ARG;
    if (numel < 0) return NF4DQ_ERR_ARG;
    if (numel == 0) return NF4DQ_OK;
    if (!packed || !out || !a2) return NF4DQ_ERR_ARG;
    if (blocksize < 64 || (blocksize & (blocksize - 1))) return NF4DQ_ERR_ARG;
    const int64_t nblk = (numel + blocksize - 1) / blocksize;
    if (nb < nblk) return NF4DQ_ERR_SHAPE;
    if (!single) {
        if (!a1 || !code2) return NF4DQ_ERR_ARG;
        if (blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1))) return NF4DQ_ERR_ARG;
        if (n2 < (nblk + blocksize2 - 1) / blocksize2) return NF4DQ_ERR_SHAPE;
    }
    const int mode = single ? kBnbSingle : kBnb;
    if (numel % 8 == 0 && nblk < kMaxFlatBlocks && blocksize <= (1 << 28) && aligned(packed, 4) && aligned(out, 16)) {
        // the stream as one matrix of rows of kPieceBytes / 2 packed bytes (a
        // multiple of every block's byte count): pieces exactly as above
        const int64_t nbytes = numel / 2;
        const int64_t row = nbytes < kPieceBytes ? nbytes : kPieceBytes / 2;
        Desc d{};
        d.packed = reinterpret_cast<const uint32_t*>(packed);
        d.a1 = a1;
        d.a2 = a2;
        d.code2 = code2;
        d.out = reinterpret_cast<u32x4*>(out);
        d.offset = offset;
        d.blk_shift = (uint32_t)ilog2((uint64_t)blocksize / 2);
        d.blk2_shift = single ? 0u : (uint32_t)ilog2((uint64_t)blocksize2);
        if (nbytes < kPieceBytes) {
            Batch<1> b{};
            b.d[0] = d;
            b.d[0].nbytes = (uint32_t)nbytes;
            b.count = 1;
            b.total_tiles = (uint32_t)((nbytes + 1023) / 1024);
            return launch_flat_batch(b, dtype, mode, kDefaultCfg, st);
        }
        Batch<NF4DQ_BATCH_MAX> b{};
        const int64_t ob = dtype == NF4DQ_F32 ? 8 : 4;  // output bytes per packed byte
        for (int64_t p0 = 0; p0 < nbytes; p0 += row) {
            Desc x = d;
            const int64_t len = nbytes - p0 < row ? nbytes - p0 : row;
            x.packed = reinterpret_cast<const uint32_t*>(packed + p0);
            x.out = reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(out) + p0 * ob);
            x.nbytes = (uint32_t)len;
            x.blk_base = (uint32_t)(p0 >> d.blk_shift);
            x.tile_begin = b.total_tiles;
            b.d[b.count++] = x;
            b.total_tiles += (uint32_t)((len + 1023) / 1024);
            if (b.count == NF4DQ_BATCH_MAX) {
                const int rc = launch_flat_batch(b, dtype, mode, kDefaultCfg, st);
                if (rc) return rc;
                b.count = 0;
                b.total_tiles = 0;
            }
        }
        return b.count ? launch_flat_batch(b, dtype, mode, kDefaultCfg, st) : NF4DQ_OK;
    }
    BnbBytesArgs A{};
    A.packed = packed;
    A.a1 = a1;
    A.code2 = code2;
    A.a2 = a2;
    A.out = out;
    A.offset = offset;
    A.numel = numel;
    A.blk_shift_elems = ilog2((uint64_t)blocksize);
    A.blk2_shift = single ? 0 : ilog2((uint64_t)blocksize2);
    A.single = single ? 1 : 0;
    const unsigned g = rows_grid((numel + 1) / 2);
    if (dtype == NF4DQ_BF16) hipLaunchKernelGGL((nf4_bnb_bytes_kernel<NF4DQ_BF16>), dim3(g), dim3(kWg), 0, st, A);
    else if (dtype == NF4DQ_F16) hipLaunchKernelGGL((nf4_bnb_bytes_kernel<NF4DQ_F16>), dim3(g), dim3(kWg), 0, st, A);
    else hipLaunchKernelGGL((nf4_bnb_bytes_kernel<NF4DQ_F32>), dim3(g), dim3(kWg), 0, st, A);
    return hip_rc(hipGetLastError());
}

int nf4_dequant_bnb(const uint8_t* packed, const uint8_t* absmax_q, int64_t nb, const float* code2,
                    const float* absmax2, int64_t n2, float offset, void* out, int32_t out_dtype, int64_t numel,
                    int32_t blocksize, int32_t blocksize2, void* hip_stream) {
    return bnb_common(packed, absmax_q, nb, code2, absmax2, n2, offset, out, out_dtype, numel, blocksize, blocksize2,
                      false, reinterpret_cast<hipStream_t>(hip_stream));
}

int nf4_dequant_bnb_single(const uint8_t* packed, const float* absmax, int64_t nabs, void* out, int32_t out_dtype,
                           int64_t numel, int32_t blocksize, void* hip_stream) {
    return bnb_common(packed, nullptr, nabs, nullptr, absmax, 0, 0.0f, out, out_dtype, numel, blocksize, 1, true,
                      reinterpret_cast<hipStream_t>(hip_stream));
}

const char* nf4_strerror(int code) {
    switch (code) {
        case NF4DQ_OK: return "ok";
        case NF4DQ_ERR_ARG: return "invalid argument (null pointer, dtype or negative size)";
        case NF4DQ_ERR_SHAPE: return "shape mismatch (packed weight / absmax cannot be viewed as the reference does)";
        case NF4DQ_ERR_TOO_LARGE: return "matrix too large for one launch";
        case NF4DQ_ERR_SPLITK_TIMEOUT:
            return "fused GEMM split-K hand-off timed out (some outputs are NaN; workspace re-zeroed)";
        default: break;
    }
    if (code >= NF4DQ_ERR_HIP_BASE) return hipGetErrorString((hipError_t)(code - NF4DQ_ERR_HIP_BASE));
    return "unknown error";
}

const char* nf4_version(void) { return "nf4dq 0.2.0 gfx950"; }

#if NF4_FLAT_STAMPS
// Diagnostic build only: where the flat kernel writes its per-wave stamps.
void nf4_dbg_set_stamps(void* buf) { g_stamps = reinterpret_cast<unsigned long long*>(buf); }
#endif

}  // extern "C"
