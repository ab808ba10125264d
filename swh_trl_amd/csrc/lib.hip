// Library identity and status strings of the swh_trl_amd C-ABI.
#include "common.hpp"

extern "C" const char *swh_version(void) { return "swh_trl_amd 0.1.0 (gfx950)"; }

extern "C" const char *swh_status_string(int status) {
    switch (status) {
    case SWH_OK: return "ok";
    case SWH_E_ARG: return "invalid argument";
    case SWH_E_LAUNCH: return "kernel launch failed";
    case SWH_E_DTYPE: return "unsupported dtype";
    default: return "unknown status";
    }
}
