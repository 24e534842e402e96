// The NF4_ABL_* hook definitions of the ablation builds (tools only), selected by
// -DABL_<part>; included by tools/gemm_ablate.hip and, for stamped ablations, by
// tools/gemm_stamps.hip.  Without any ABL_* macro it defines nothing.
#pragma once
#if defined(ABL_NTW)  // weight loads with the nt (streaming) policy, as the flat dequant kernel's
#define NF4_ABL_WLOAD(rsrc_, off_) __builtin_amdgcn_raw_buffer_load_b128((rsrc_), (off_), 0, 2)
#endif
// (ABL_CONT, round 6: one lookup pipeline across chunks -- measured slower at ring depth 2,
// profiles/r06/gemm/s6_cont_pipeline_ab.jsonl; the variant is in git history at e7f9535)
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
#if defined(ABL_NOXR)  // the persistent / streaming body's x fragments from registers: one constant
// fragment, materialised once outside the loops (no LDS read, no VALU per step; wrong results)
#define NF4_ABL_XFRAG(smem_, off_) (u32x4{0x3F803F80u, 0x3E803F00u, 0x3F803E80u, 0x3F003F80u})
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

