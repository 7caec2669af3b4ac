// ak_k_switches.hip — kernel instantiations for one op (a separate TU so hipcc builds ops in parallel).
#include "ak_internal.h"

namespace ak {

int launch_switches(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (flags) {
        case -1: return launch_rows<OP_SWITCHES, -1>(w, a, out_offs, st);
        case 0: return launch_rows<OP_SWITCHES, 0>(w, a, out_offs, st);
        case 1: return launch_rows<OP_SWITCHES, 1>(w, a, out_offs, st);
        case 2: return launch_rows<OP_SWITCHES, 2>(w, a, out_offs, st);
        case 3: return launch_rows<OP_SWITCHES, 3>(w, a, out_offs, st);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "switches: unsupported flags");
}

}  // namespace ak
