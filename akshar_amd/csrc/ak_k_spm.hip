// ak_k_spm.hip — kernel instantiations for one op (a separate TU so hipcc builds ops in parallel).
#include "ak_internal.h"

namespace ak {

// SPM ids per row <= 3 * raw bytes + 3: NFC at most triples a char's UTF-8 bytes (UAX #15), every
// id covers >= 1 normalized byte (byte fallback: exactly 1), and each "▁" (3 bytes) stands for
// >= 1 raw space byte except the dummy prefix (+3). One staged pass, no count pass.
constexpr uint32_t SPM_MUL = 3, SPM_ADD = 4;

int launch_spm(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (flags) {
        case 0: return launch_rows_staged<OP_SPM, 0>(w, a, out_offs, st, SPM_MUL, SPM_ADD);
        case 1: return launch_rows_staged<OP_SPM, 1>(w, a, out_offs, st, SPM_MUL, SPM_ADD);
        case 2: return launch_rows_staged<OP_SPM, 2>(w, a, out_offs, st, SPM_MUL, SPM_ADD);
        case 3: return launch_rows_staged<OP_SPM, 3>(w, a, out_offs, st, SPM_MUL, SPM_ADD);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "spm: unsupported flags");
}

}  // namespace ak
