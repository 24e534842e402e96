// A/B variants of the flat dequant kernel (tools only; never in the product library).
// Sets the NF4_DQ_* hooks of nf4_dequant.hip from -DDQV_* values and includes the
// product source; tools/Makefile `dqv` builds one library per named variant (its
// DQV flags in the Makefile's table), linked with tools/gemm_stub.cpp (the GEMM entry
// points as ERR_ARG stubs, so a variant library stays small) and the product's
// host-CPU object into tools/_build/libnf4dq_dqv_<name>.so, timed against the
// product by tools/cache_ab.py --libs in the regime where the weights stream from HBM.
//   DQV_WG=n   waves per workgroup (product 4)
//   DQV_U=n    packed dwords per lane per tile (product 4)
//   DQV_LD=p   cache-policy bits of the packed-weight loads (product 2 = nt; 16 = sc1, 1 = sc0, 0 = default)
//   DQV_ST=p   cache-policy bits of the output stores (product 18 = sc1 + nt)
//   DQV_SF=1   a tile's scale loads issued before its packed loads
//   DQV_SNT=1  the absmax / nested-scale gathers with the nt policy
//   DQV_NOSCALE=1  ablation: no scale loads (wrong results; timing only)
// Round 5 also measured store delays, scale-gather buffer loads / policies, a table decode
// without the code table and its barrier, and synchronised stores through hooks removed
// after measurement (profiles/r05/; the hooks are in git history at 914c6b8), and scale-index shortcuts and
// gather delays (at 414c083), bitsandbytes-mode code-table loads and gather
// delays (at 99ed841), and the chunk kernel's barrier / scale-gather placements (at 1601634).
//   DQV_SINGLE=1   one-tile waves skip the pipelined loop
//   DQV_FE=n   chunk kernel's LDS-staged flush (NF4_DQ_FLUSH_EDGE: 1 edge lines default policy,
//              2 no end-piece element stores (timing only), 3 all flush stores default policy);
//              measured in round 6 (profiles/r06/chunk/s3_flush_variants.jsonl), the hook removed
//              after measurement (it is in git history at effdce7)
//   DQV_LD64=1 the piece kernel's 8-byte packed loads (NF4_DQ_PIECE_LD64): 5-13 % slower in
//              round 6 (profiles/r06/chunk/s14_piece_ld64_ab.jsonl); the hook removed after
//              measurement (in git history at the commit that adds that file)
//   DQV_F32ST=p  cache-policy bits of the chunk kernel's fp32 half-chunk stores (padded rows):
//              0 (default policy) 18.3 us at padded 4096^2 fp32 against 57.2 (sc1 + nt) and 41.5
//              (sc1), round 6 (profiles/r06/chunk/s19_f32_half_store_policy.jsonl); 0 is now the
//              product's and the hook is gone
//   DQV_DEC=n  16-bit output decode (NF4_DQ_DECODE: 0 per-nibble lookup + multiply, 1 per-block LDS table)
#ifdef DQV_WG
#define NF4_DQ_FLAT_WAVES DQV_WG
#endif
#ifdef DQV_U
#define NF4_DQ_U DQV_U
#endif
#ifdef DQV_LD
#define NF4_DQ_AUX_LOAD DQV_LD
#endif
#ifdef DQV_ST
#define NF4_DQ_AUX_STORE DQV_ST
#endif
#ifdef DQV_SF
#define NF4_DQ_SCALE_FIRST DQV_SF
#endif
#ifdef DQV_SNT
#define NF4_DQ_SCALE_NT DQV_SNT
#endif
#ifdef DQV_FE  // chunk kernel's staged flush (NF4_DQ_FLUSH_EDGE), round 6
#define NF4_DQ_FLUSH_EDGE DQV_FE
#endif

#ifdef DQV_NOSCALE
#define NF4_DQ_ABL_NOSCALE DQV_NOSCALE
#endif
#ifdef DQV_SINGLE
#define NF4_DQ_SINGLE_FAST DQV_SINGLE
#endif
#ifdef DQV_DEC
#define NF4_DQ_DECODE DQV_DEC
#endif

#include "../nf4_triton_dequantization_amd/csrc/nf4_dequant.hip"
