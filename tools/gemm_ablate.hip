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

#include "gemm_ablate_hooks.h"
// the product's fused-GEMM sources, all in this one translation unit
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_k128.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_persist.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_stream.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_xr.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_xs.hip"
