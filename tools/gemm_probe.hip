// Instrumented build of the decode kernels for tools/gemm_probe.py: the same
// source with per-workgroup phase timestamps (SWH_GEMM_TRACE_ON).  Tuning aid only.
#define SWH_GEMM_TRACE_ON 1
#include "../swh_trl_amd/csrc/decode.hip"

extern "C" int swh_probe_set_trace(unsigned long long *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(swh::g_gemm_trace), &p, sizeof(p)) == hipSuccess ? 0 : -2;
}
