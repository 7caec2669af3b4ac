// ak_k_normalize.hip — kernel instantiations for one op (a separate TU so hipcc builds ops in parallel).
#include "ak_internal.h"

namespace ak {

// normalized UTF-8 bytes per row <= 3 * raw bytes (ak_normalize_cap: NFC at most triples a char's
// bytes, the lower / allowlist map never grows one past that). One staged pass, no count pass.
constexpr uint32_t STAGE_MUL = 3, STAGE_ADD = 1;

int launch_normalize(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (flags) {
        case 0: return launch_rows_staged<OP_NORMALIZE, 0>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        case 1: return launch_rows_staged<OP_NORMALIZE, 1>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        case 2: return launch_rows_staged<OP_NORMALIZE, 2>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        case 3: return launch_rows_staged<OP_NORMALIZE, 3>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "normalize: unsupported flags");
}

}  // namespace ak
