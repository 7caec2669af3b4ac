// ak_k_normalize_st.hip — ak_normalize with AK_NORM_STAGES: the step subsets of normalize_text
// that no flags value names (normalize_unicode alone is flags 0, normalize_text flags 0..3).
#include "ak_internal.h"

namespace ak {

constexpr uint32_t ST_MUL = 3, ST_ADD = 1;  // as ak_k_normalize.hip: NFC at most triples a row's bytes

template <int ST>
static int run_st(AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    return launch_rows_staged<OP_NORMALIZE, AK_NORM_STAGES | ST>(w, a, out_offs, st, ST_MUL, ST_ADD);
}

int launch_normalize_stages(int stages, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    switch (stages) {
        case 0: return run_st<0>(w, a, out_offs, st);
        case 2: return run_st<2>(w, a, out_offs, st);
        case 4: return run_st<4>(w, a, out_offs, st);
        case 6: return run_st<6>(w, a, out_offs, st);
        case 8: return run_st<8>(w, a, out_offs, st);
        case 10: return run_st<10>(w, a, out_offs, st);
        case 12: return run_st<12>(w, a, out_offs, st);
        case 14: return run_st<14>(w, a, out_offs, st);
        case 5: return run_st<5>(w, a, out_offs, st);
        case 7: return run_st<7>(w, a, out_offs, st);
        case 9: return run_st<9>(w, a, out_offs, st);
        case 11: return run_st<11>(w, a, out_offs, st);
        default: break;
    }
    return set_error(AK_ERR_UNSUPPORTED, "normalize: unsupported stage mask");
}

}  // namespace ak
