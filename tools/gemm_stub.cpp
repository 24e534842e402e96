// The fused-GEMM entry points of include/nf4_dequant.h as stubs (tools only): the
// dequant A/B libraries (tools/dq_variants.hip) export every declared symbol, so
// nf4_triton_dequantization_amd/_lib.py binds them, without carrying the GEMM object.
#include "../include/nf4_dequant.h"

extern "C" {
size_t nf4_gemm_workspace_bytes(int64_t, int64_t, int64_t) { return 0; }
size_t nf4_gemm_workspace_bytes_cfg(int64_t, int64_t, int64_t, const nf4_gemm_cfg*) { return 0; }
size_t nf4_gemm_grouped_workspace_bytes(int64_t, int64_t, const nf4_gemm_mat*, int32_t, const nf4_gemm_cfg*) {
    return 0;
}
int nf4_gemm_ref(const void*, int64_t, const uint8_t*, int64_t, const uint8_t*, int64_t, const float*, int64_t, void*,
                 int32_t, int64_t, int64_t, void*, size_t, void*) {
    return NF4DQ_ERR_ARG;
}
int nf4_gemm_ref_cfg(const void*, int64_t, const uint8_t*, int64_t, const uint8_t*, int64_t, const float*, int64_t,
                     void*, int32_t, int64_t, int64_t, void*, size_t, const nf4_gemm_cfg*, void*) {
    return NF4DQ_ERR_ARG;
}
int nf4_gemm_ref_grouped(const void*, int64_t, int64_t, const nf4_gemm_mat*, int32_t, int32_t, void*, size_t,
                         const nf4_gemm_cfg*, void*) {
    return NF4DQ_ERR_ARG;
}
int nf4_gemm_check_workspace(void*, size_t, void*) { return NF4DQ_ERR_ARG; }
}
