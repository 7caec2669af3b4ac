// ak_k_segment.hip — kernel instantiations for one op (a separate TU so hipcc builds ops in parallel).
#include "ak_internal.h"

namespace ak {

// clusters per row <= code points after normalization <= 3 * raw bytes (NFC at most triples the
// code points of a char, every raw code point has >= 1 byte). One staged pass, no count pass.
constexpr uint32_t STAGE_MUL = 3, STAGE_ADD = 1;

int launch_segment(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (flags) {
        case -1: return launch_rows_staged<OP_SEGMENT, -1>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        case 0: return launch_rows_staged<OP_SEGMENT, 0>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        case 1: return launch_rows_staged<OP_SEGMENT, 1>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        case 2: return launch_rows_staged<OP_SEGMENT, 2>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        case 3: return launch_rows_staged<OP_SEGMENT, 3>(w, a, out_offs, st, STAGE_MUL, STAGE_ADD);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "segment: unsupported flags");
}

}  // namespace ak
