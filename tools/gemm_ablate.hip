// Ablation builds of the pair-table decode-GEMM kernels (tools only; timing,
// never correctness).  Redefines one of the NF4_ABL_* hooks of nf4_gemm.hip (selected
// by -DABL_<part>) and includes the product source; tools/Makefile `ablate` links
// each variant with the product's dequant and host objects into
// tools/_build/libnf4dq_abl_<part>.so, timed by tools/gemm_ab.py.
//   ABL_NOLUT   codes made from the address bits instead of the pair-table read
//   ABL_NOWLOAD weight "loads" made from their offsets (no memory traffic)
//   ABL_NOMMA   no MFMAs (operands kept alive)
//   ABL_NORED   no in-LDS reduction of the K-partial tiles (no per-strip barriers)
//   ABL_NOHAND  no split-K hand-off (no slab stores, tickets or last-arriver sums)
//   ABL_NOX     register-resident kernel: no global loads of the x fragments
//   ABL_NOSCALE register-resident kernel: no absmax byte / nested scale gathers
//   ABL_NORING  ABL_NOWLOAD + ABL_NOSCALE: the ring issues no memory operation
//   ABL_L2WIN   weight loads folded into a 256 KiB window (L2-resident, same instructions)
//   ABL_SKELETON ABL_NORING + ABL_NOLUT + ABL_NOMMA: control flow, x staging, tables, VALU
//   ABL_PAIR    persistent kernel: two ring slots decoded step-interleaved (variant: correct results)
//   ABL_EMPTY   persistent kernel: returns at entry (the launch of its grid, nothing else)
//   ABL_NOLOOP  persistent kernel: no chunk loop (x staging, tables, outputs: the fixed cost)
//   ABL_NTW     weight loads with the nt policy (a variant, not an ablation: correct results)
//   ABL_DROPSLICE  128-deep kernel: K slice 1 withholds its split-K partials (takes its
//               ticket all the same), so the reducer's bounded poll gives up: proves the
//               workspace error word fires (tools/splitk_timeout_probe.py, one run)
#include <hip/hip_runtime.h>

#if defined(ABL_NTW)  // weight loads with the nt (streaming) policy, as the flat dequant kernel's
#define NF4_ABL_WLOAD(rsrc_, off_) __builtin_amdgcn_raw_buffer_load_b128((rsrc_), (off_), 0, 2)
#endif
#if defined(ABL_PAIR)  // a variant, not an ablation: correct results
#define NF4_PERSIST_PAIR 1
#endif
#if defined(ABL_EMPTY)
#define NF4_ABL_ENTRY_RETURN 1
#endif
#if defined(ABL_NOLOOP)
#define NF4_ABL_LOOP_ON 0
#endif
#if defined(ABL_DROPSLICE)
#define NF4_ABL_KEEP_SLICE(ks_) ((ks_) != 1u)
#endif

#if defined(ABL_SKELETON)  // the ring's memory operations, the lookups and the MFMAs all removed
#define ABL_NORING
#define ABL_NOLUT
#define ABL_NOMMA
#endif
#if defined(ABL_NORING)  // no memory traffic in the ring at all
#define ABL_NOWLOAD
#define ABL_NOSCALE
#endif
#if defined(ABL_NOWLOAD) || defined(ABL_NOSCALE)  // the ring issues fewer loads per slot
#define NF4_ABL_RING_FULL 0
#endif
#if defined(ABL_NOLUT)
#define NF4_ABL_LOOKUP(pt_, addr_, wd_) \
    (f32x2{__uint_as_float(((addr_) & 0xFFFFu) | 0x3F000000u), __uint_as_float(((wd_) & 0xFFFFu) | 0x3E000000u)})
#endif
#if defined(ABL_NOWLOAD)
#define NF4_ABL_WLOAD(rsrc_, off_) (u32x4{(off_), (off_) * 3u, (off_) ^ 0x5A5A5A5Au, (off_) + 0x01010101u})
#elif defined(ABL_L2WIN)  // weight loads folded into a 256 KiB window per weight: L2 hits, same instructions
#define NF4_ABL_WLOAD(rsrc_, off_) __builtin_amdgcn_raw_buffer_load_b128((rsrc_), (off_) & 0x8003FFF0u, 0, 0)
#endif
#if defined(ABL_NOSCALE)  // (the persistent kernel's 8/16-byte scale loads too)
#define NF4_ABL_PLOAD_FAKE 1
#endif
#if defined(ABL_NOSCALE)  // absmax byte / nested scale from the offset (no gather)
#define NF4_ABL_SLOAD(rsrc_, off_, b8_) ((b8_) ? (((off_) * 37u) & 0x7Fu) | 1u : 0x3C000000u | ((off_) & 0xFFFFu))
#endif
#if defined(ABL_NOX)
#define NF4_ABL_X_ON 0
#endif
#if defined(ABL_NOMMA)
#define NF4_ABL_MMA_ON 0
#define NF4_ABL_RED_ON 1
#define NF4_ABL_HANDOFF_ON 1
#elif defined(ABL_NORED)
#define NF4_ABL_MMA_ON 1
#define NF4_ABL_RED_ON 0
#define NF4_ABL_HANDOFF_ON 1
#elif defined(ABL_NOHAND)
#define NF4_ABL_MMA_ON 1
#define NF4_ABL_RED_ON 1
#define NF4_ABL_HANDOFF_ON 0
#endif

// the product's fused-GEMM sources, all in this one translation unit
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_k128.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_persist.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_sk.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_stream.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_xr.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_xs.hip"
