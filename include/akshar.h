/*
 * akshar.h — C-ABI of the MI355X batch tokenization engine (libakshar: akshar_amd/_akshar_hip.so).
 *
 * The reference (Bhasha-Open/Akshar, pure Python) has no FFI: its boundary is the Python API
 * (src/akshar/tokenizer.py:18-288, src/akshar/__init__.py:12-109) plus a duck-typed engine seam
 * `self.model.encode(str).ids` / `self.model.EncodeAsIds(str)` (tokenizer.py:153-156,190-193).
 * Each entry point below replaces one reference interface, batched: rows are packed UTF-8 in one
 * byte buffer with u64 row offsets, every output is a packed buffer plus u64 row offsets.
 *
 * Conventions
 *  - Every call returns an int status (AK_OK or a negative AK_ERR_*); ak_last_error() returns a
 *    thread-local message for the last failure on the calling thread.
 *  - All array arguments of the batch calls are DEVICE pointers (hipMalloc / torch CUDA tensors)
 *    on the current HIP device; `stream` is a hipStream_t (NULL = default stream). Batch calls
 *    only enqueue work: results are valid after the stream is synchronized.
 *  - Input: `in` holds offs[n] bytes (offs[0] == 0, offs non-decreasing). Each row is one string
 *    of the reference API. The buffer must stay readable through offs[n] rounded up to 16 bytes (rows are
 *    read in aligned 16-byte blocks).
 *  - Output sizing: callers pass a capacity `cap` (elements). out_offs[0..n] is always written;
 *    the total is out_offs[n]. If out_offs[n] > cap, the call still returns AK_OK but the output
 *    elements are incomplete: re-run with cap >= out_offs[n] (the bound helpers below give caps
 *    that are always sufficient).
 *  - row_status (optional, u8[n], may be NULL): bit 0 = row had invalid UTF-8 (decoded as U+FFFD
 *    per byte). Bit 2 (AK_ROW_LIMIT) is only ever set together with an engine-bug error from
 *    ak_ws_check(): no row length is rejected (see "Row lengths").
 *  - Row lengths: there is no per-row limit. Rows run in up to three tiers: the fast kernels
 *    (small private buffers), the slow tier (per-thread pool regions of AK_SLOW_TIER_ENTRIES code
 *    points per NFC segment / symbols per BPE pre-token or SentencePiece word), and the huge tier,
 *    whose pool is sized from the longest row past the slow tier (one extra host read-back; about
 *    300 bytes of device memory per input byte of that row). A call whose huge tier cannot be
 *    allocated fails with AK_ERR_NOMEM; it never returns a short or empty row.
 *  - Models and workspaces are not thread-safe for concurrent calls on different streams with the
 *    same workspace; models are immutable after creation and may be shared.
 */
#ifndef AKSHAR_H
#define AKSHAR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AK_OK 0
#define AK_ERR_ARG (-1)
#define AK_ERR_HIP (-2)
#define AK_ERR_UNSUPPORTED (-3)
#define AK_ERR_NOMEM (-4)

/* normalize_text flags (normalize.py:117 `normalize_text(text, normalize_roman, clean_hinglish)`) */
#define AK_NORM_LOWER 1 /* normalize_roman=True: 'LATIN' in name(c) -> c.lower()  (normalize.py:21-45) */
#define AK_NORM_CLEAN 2 /* clean_hinglish=True: allowlist filter + elongation collapse (:92-114) */
#define AK_NORM_DEFAULT (AK_NORM_LOWER | AK_NORM_CLEAN)
#define AK_RAW (-1)     /* segment/switches on the raw row (the free functions on unnormalized text) */

/* ak_normalize only: AK_NORM_STAGES | any AK_ST_* runs exactly the selected steps of normalize_text,
 * in its order, each of which the reference also exports on its own (normalize.py:13-114):
 *   normalize_unicode  AK_ST_NFC          semantic_normalize AK_ST_LOWER
 *   filter_garbage     AK_ST_FILTER       remove_elongations AK_ST_ELONG
 *   normalize_hinglish AK_ST_FILTER | AK_ST_ELONG   (:110-114; no NFC, no lowercasing)
 * AK_NORM_STAGES | AK_ST_NFC | AK_ST_LOWER | AK_ST_FILTER | AK_ST_ELONG == AK_NORM_DEFAULT. */
#define AK_NORM_STAGES 16
#define AK_ST_NFC 1    /* unicodedata.normalize('NFC') (:13-18) */
#define AK_ST_LOWER 2  /* 'LATIN' in name(c) -> c.lower() (:21-45) */
#define AK_ST_FILTER 4 /* allowlist filter (:92-107) */
#define AK_ST_ELONG 8  /* re.sub(r'(.)\1{2,}', r'\1') (:48-56) */

/* per-row status bits */
#define AK_ROW_BAD_UTF8 1u
#define AK_ROW_LIMIT 4u

/* per-thread capacity of the slow tier (code points of one NFC segment, symbols of one BPE
 * pre-token, chars of one SentencePiece word); longer ones run in the huge tier */
#define AK_SLOW_TIER_ENTRIES 4096

typedef struct ak_bpe ak_bpe; /* device-resident BPE model (HF tokenizers models.BPE) */
typedef struct ak_spm ak_spm; /* device-resident SentencePiece unigram model */
typedef struct ak_ws ak_ws;   /* device scratch, grows on demand; one per stream */

const char *ak_last_error(void);
int ak_version(void);
/* Device self-test of the wave64 primitives the tile kernels rely on (DPP prefix scan, readlane
 * broadcast, ballot): AK_OK, or AK_ERR_HIP with the first mismatch in ak_last_error(). */
int ak_selftest(void);

int ak_ws_create(ak_ws **out);
void ak_ws_free(ak_ws *ws);
/* Kernel choice for this workspace's calls with the normalize_text defaults (flags 3: BPE and
 * SentencePiece encodes, normalize, segment / switches of normalized rows, analyze): path 1 =
 * tile-cooperative single pass (default; a wave packs up to tile_rows rows, 1..16, default 16,
 * into each tile, as many as fit its byte buffer), 0 = one lane per row (the staged row kernels). */
int ak_ws_set_tiling(ak_ws *ws, int bpe_path, int tile_rows);
/* Synchronous health check after a batch: AK_ERR_HIP if the last call flagged an internal
 * overflow (a row producing more output than its staging slot bound, or overflowing the huge
 * tier; never observed). */
int ak_ws_check(ak_ws *ws);

/* Replaces Tokenizer.from_file(path) (tokenizer.py:96-97) for the model cli.py:276-299 trains:
 * NFKC -> Whitespace -> BPE(unk_token=None) -> "<s> $A </s>".
 * single_cp/single_id: the single-code-point vocab entries; merges: n_merges x {left, right, new}
 * in rank order (rank = row index); bos/eos: the template's special ids. Host pointers. */
int ak_bpe_create(uint32_t n_single, const uint32_t *single_cp, const uint32_t *single_id,
                  uint32_t n_merges, const uint32_t *merges, uint32_t bos, uint32_t eos, ak_bpe **out);
void ak_bpe_free(ak_bpe *m);
/* The tile path's pre-token result cache, built by ak_bpe_create (HF BPE's per-word cache,
 * tokenizer.py:96-97,193, made exact at load: keys are the char-id sequences of merged tokens whose
 * merge_all is that one id). info[0] table slots (0 = no cache: not a tile-path model, or AK_PTC=0
 * in the environment), [1] keys found, [2] keys stored, [3] merged-token sequences whose merge_all is
 * not one id (never stored). */
int ak_bpe_cache_info(const ak_bpe *m, uint64_t info[4]);
/* The tokenizer's added tokens (tokenizer.json "added_tokens": <pad> <unk> <s> </s> <mask> for
 * cli.py:283-285), all normalized=false / lstrip=rstrip=single_word=false: HF's AddedVocabulary
 * splits the text it receives on them (leftmost-longest) BEFORE the NFKC normalizer, each match
 * becoming its id and each piece between encoded on its own. Only reachable with
 * clean_hinglish=False (the allowlist drops '<' '>' '/'); a token made only of allowlisted chars is
 * AK_ERR_UNSUPPORTED. n tokens <= AK_MAX_ADDED, each 1..16 code points: cps packed with
 * cp_offs[n+1]. Host pointers; replaces any previous set. */
#define AK_MAX_ADDED 64
int ak_bpe_set_added(ak_bpe *m, uint32_t n, const uint32_t *cps, const uint32_t *cp_offs, const uint32_t *ids);

/* Replaces SentencePieceProcessor.Load(path) (tokenizer.py:88-90) for the unigram model
 * cli.py:232-248 trains (identity normalizer, byte_fallback). pieces: n UTF-8 strings packed in
 * piece_bytes with piece_offs[n+1]; scores float[n]; types u8[n] (sentencepiece_model.proto
 * enum: 1 NORMAL 2 UNKNOWN 3 CONTROL 4 USER_DEFINED 5 UNUSED 6 BYTE); byte_ids[256]: ids of
 * <0x00>..<0xFF>. Host pointers. */
int ak_spm_create(uint32_t n, const uint8_t *piece_bytes, const uint64_t *piece_offs, const float *scores,
                  const uint8_t *types, int32_t unk_id, const int32_t *byte_ids, ak_spm **out);
void ak_spm_free(ak_spm *m);
/* The tile path's word cache, built by ak_spm_create when AK_SWC=1 is in the environment (off by
 * default: measured slower): the base-0 lattice solution (pieces and the smallest
 * winning margin) of every "▁"-initial piece string, solved at load; a hit is accepted under the
 * same rounding-bound test as a solved word. info[0] table slots (0 = no cache), [1] words found,
 * [2] words stored, [3] words whose solution holds an unknown char or more than 6 pieces (never
 * stored). */
int ak_spm_cache_info(const ak_spm *m, uint64_t info[4]);

/* Model files read inside the library (host code, no GPU needed to parse): a caller over the
 * C-ABI needs no tokenizer.json / protobuf parser of its own. Same acceptance rules as
 * ak_bpe_create / ak_spm_create above (and akshar_amd/models.py).
 * ak_bpe_load: HF tokenizer.json -> ak_bpe_create + ak_bpe_set_added + ak_bpe_set_vocab
 *   (replaces Tokenizer.from_file, tokenizer.py:96-97).
 * ak_spm_load: SentencePiece .model (ModelProto wire format) -> ak_spm_create
 *   (replaces SentencePieceProcessor.Load, tokenizer.py:88-90).
 * ak_model_load: model_type "bpe" (-> ak_bpe*) or "sentencepiece" (-> ak_spm*), the reference's
 *   aksharTokenizer(model_path, model_type) choice (tokenizer.py:54-102); ak_model_free likewise.
 *   The library keeps a set of its live handles: ak_model_free of a pointer that is not one (never
 *   created, or already freed) sets AK_ERR_ARG's message and touches nothing.
 * ak_model_info (parse only, no device): info[0] vocab / piece count, BPE: [1] single-char
 *   entries, [2] merges, [3] bos, [4] eos, [5] added tokens; SPM: [1] unk id; [7] a 64-bit FNV-1a
 *   of every array the loader would pass to the create calls, in their argument order. */
int ak_bpe_load(const char *path, ak_bpe **out);
int ak_spm_load(const char *path, ak_spm **out);
int ak_model_load(const char *path, const char *model_type, void **out);
void ak_model_free(void *h, const char *model_type);
int ak_model_info(const char *path, const char *model_type, uint64_t info[8]);

/* normalize_text(text, normalize_roman, clean_hinglish) (normalize.py:117-148) per row, flags
 * 0..3; or AK_NORM_STAGES | AK_ST_* for any subset of its steps (above).
 * out: UTF-8 bytes; a sufficient cap is ak_normalize_cap(). */
int ak_normalize(ak_ws *ws, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n, uint8_t *out,
                 uint64_t cap, uint64_t *out_offs, uint8_t *row_status, void *stream);

/* segment_akshars(text, matras) (segment.py:40-125) per row: cluster END indices (code points,
 * relative to the row) of the normalized row (flags >= 0, as tokenize() without a model,
 * tokenizer.py:144-151) or of the raw row (flags == AK_RAW). */
int ak_segment(ak_ws *ws, int flags, int matras, const uint8_t *in, const uint64_t *offs, uint64_t n,
               uint32_t *ends, uint64_t cap, uint64_t *out_offs, uint8_t *row_status, void *stream);

/* detect_code_switches(text) (segment.py:150-201) per row: run END indices (code points) and
 * labels (0 other, 1 devanagari, 2 roman, 255 None = all-neutral row). */
int ak_switches(ak_ws *ws, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n, uint32_t *ends,
                uint8_t *labels, uint64_t cap, uint64_t *out_offs, uint8_t *row_status, void *stream);

/* The front half of aksharTokenizer.explain(text) / tokenize(text, return_metadata=True)
 * (tokenizer.py:248-276, :146-147; segment.py:210-236), fused into ONE pass per row:
 * norm = normalize_text(text, flags) as UTF-8 (like ak_normalize), and on that normalized text
 * segment_akshars(norm, matras) cluster ENDs (like ak_segment with AK_RAW on norm) and
 * detect_code_switches(norm) run ENDs + labels (like ak_switches with AK_RAW on norm).
 * Three outputs, each with its own capacity and u64[n+1] offsets ([n] = required total). */
int ak_analyze(ak_ws *ws, int flags, int matras, const uint8_t *in, const uint64_t *offs, uint64_t n,
               uint8_t *norm, uint64_t norm_cap, uint64_t *norm_offs, uint32_t *clusters, uint64_t cl_cap,
               uint64_t *cl_offs, uint32_t *runs, uint8_t *labels, uint64_t run_cap, uint64_t *run_offs,
               uint8_t *row_status, void *stream);

/* aksharTokenizer(model, "bpe").encode(text) (tokenizer.py:167-193): normalize_text(flags) then
 * the HF pipeline; ids include <s> ... </s>. Any flags 0..3: with AK_NORM_CLEAN the normalized
 * text is over the allowlist (tile path for flags 3); without it (clean_hinglish=False) any text
 * reaches the tokenizer: added-token split, HF's full NFKC (Unicode 9 tables of tokenizers
 * 0.22.2) and the Whitespace pre-tokenizer over every code point, one lane per row. */
int ak_bpe_encode(const ak_bpe *m, ak_ws *ws, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n,
                  uint32_t *ids, uint64_t cap, uint64_t *out_offs, uint8_t *row_status, void *stream);

/* aksharTokenizer(model, "sentencepiece").encode(text) (tokenizer.py:167-193): normalize_text then
 * EncodeAsIds (no bos/eos). */
int ak_spm_encode(const ak_spm *m, ak_ws *ws, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n,
                  uint32_t *ids, uint64_t cap, uint64_t *out_offs, uint8_t *row_status, void *stream);

/* One string from host memory to host ids: aksharTokenizer.encode(text) as a non-Python caller binds
 * it (tokenizer.py:167-193; the FFI stub in INTEGRATION.md), for per-call latency. text: len UTF-8
 * bytes (host); ids: cap host int32 slots. The row goes through pinned staging in one
 * host->device copy, the same kernels as ak_bpe_encode / ak_spm_encode on `stream`, and one
 * device->host copy of count, error words and ids, with one stream synchronize (no read-backs in
 * between: the workspace knows the row's length). *n_ids = the id count; if it exceeds cap, nothing
 * is copied and the call returns AK_ERR_NOMEM (call again with a larger buffer). Synchronous: the
 * ids are in `ids` on return. */
int ak_bpe_encode_host(const ak_bpe *m, ak_ws *ws, int flags, const uint8_t *text, uint64_t len, int32_t *ids,
                       uint64_t cap, uint64_t *n_ids, void *stream);
int ak_spm_encode_host(const ak_spm *m, ak_ws *ws, int flags, const uint8_t *text, uint64_t len, int32_t *ids,
                       uint64_t cap, uint64_t *n_ids, void *stream);

/* Built-in kernel timing: when enabled, every batch call records HIP events around each of its
 * kernel launches on the caller's stream; ak_profile_read synchronizes the pending events and
 * returns the accumulated device time and launch count of one kernel class. */
#define AK_PROF_COUNT 0      /* fast count pass (one lane per row) */
#define AK_PROF_COUNT_SLOW 1 /* slow-path count pass (rows over the fast buffers) */
#define AK_PROF_SCAN 2       /* row counts -> row offsets (three small kernels) */
#define AK_PROF_EMIT 3       /* fast emit pass */
#define AK_PROF_EMIT_SLOW 4  /* slow-path emit pass */
#define AK_PROF_TILES 5      /* tile-cooperative BPE kernel (ids into per-unit staging runs) */
#define AK_PROF_COPY 6       /* staged ids -> final positions (tile path) */
#define AK_PROF_SPM_TILES 7  /* tile-cooperative SentencePiece kernel */
#define AK_PROF_ROW_TILES 8  /* tile-cooperative normalize / segment / switches / analyze kernel */
#define AK_PROF_FALLBACK_WAVE 9 /* fallback rows a wave each: SentencePiece redo, wave NFC + tile (BPE, SPM) */
#define AK_PROF_NKERNELS 10
/* level 0 off; 1 = HIP events around every launch (ak_profile_read; timing-neutral); 2 = also the
 * tile kernels' per-pass clocks (ak_profile_tile_passes), which instrument the kernels themselves */
int ak_profile_enable(int level);
int ak_profile_read(int kernel, double *total_ms, uint64_t *launches);
void ak_profile_reset(void);

/* Rows of the last tile-path ak_bpe_encode on this workspace that took the sequential fallback
 * kernels (NFC / HF-NFC quick check tripped, invalid UTF-8, or past the 768-byte tile buffer), and
 * how many of those needed the slow-tier pool buffers. Synchronizes the device. */
int ak_ws_fallback_rows(ak_ws *ws, uint64_t *rows, uint64_t *pool_rows);
/* The same launch in detail: [0] rows the tile kernel could not finish (SentencePiece: + the rows
 * a pooled word's margin test sent back); [1] of those, rows the tile path finished after all (NFC
 * by the fallback waves, k_bpe_nfc / k_spm_nfc; the send-backs re-encoded from the carried base by
 * k_spm_redo); [2] rows left to the one-lane row pipeline; [3] of those, rows that needed the
 * slow-tier buffers. A send-back row k_spm_redo passes on to the fallback list counts once.
 * Synchronizes. */
int ak_ws_fallback_detail(ak_ws *ws, uint64_t detail[4]);

/* Tile-kernel pass breakdown (profiling aid): device clock cycles summed over all waves for each
 * pass of the tile-cooperative BPE kernel since the last call, while profiling level 2 is on. Slots:
 * 0 byte staging, 1 decode + NFC check + map/filter, 2 fused elongation + HF NFKC + pre-tokenizer,
 * 3 pre-token cache probes, 4 pre-token start list, 5 BPE merges, 6 fallback-list append, 7 ids into the unit run +
 * counts, 8 (unused), 9 loop overhead.
 * Returns the number of slots written (0 if the tile kernel has not run), or a negative error. */
#define AK_TILE_NPASS 10
int ak_profile_tile_passes(ak_ws *ws, uint64_t *cycles, int n);
/* Event counters of the same instrumented launches (profiling level 2), reset by each call:
 * [0] BPE pre-tokens probed in the pre-token cache (slot 3 of the pass breakdown), [1] its hits,
 * [2] merge batches (64 pre-tokens a wave merges at once), [3] merge rounds, [4] lanes merging, summed
 * over rounds (lane utilisation of the merge loop = [4] / (64 [3])). SentencePiece launches: [0] / [1]
 * word-cache probes / hits, [2] word-pool batches, [3] rows redone from the carried base (in the tile,
 * or by the fallback kernels after a pooled word's margin test), [4] pooled words.
 * Returns the number of counters written (0 if no tile kernel has run), or a negative error. */
#define AK_TILE_NCOUNTERS 5
int ak_profile_tile_counters(ak_ws *ws, uint64_t *counts, int n);

/* Decode (tokenizer.py:195-219): rows of ids (u32, id_offs[n+1]) -> UTF-8 text
 * rows (out, out_offs[n+1]; out_offs[n] = required total even when cap is short).
 * ak_bpe_decode = HF Tokenizer.decode with the trained tokenizer.json (no decoder): special tokens
 * and ids outside the vocabulary are skipped, the other token strings joined by ' '. It needs the
 * vocabulary strings: ak_bpe_set_vocab (n ids, UTF-8 strings packed with tok_offs[n+1], special[n]
 * = 1 for special tokens; host pointers).
 * ak_spm_decode = SentencePieceProcessor.DecodeIds: control pieces vanish, <unk> -> " \u2047 ",
 * U+2581 -> ' ', <0xXX> byte runs reassembled as UTF-8 (invalid bytes -> U+FFFD each), leading
 * U+2581 dropped until the first non-empty piece; an id past the vocabulary is AK_ERR_ARG.
 * Device pointers; one wave per row. */
int ak_bpe_set_vocab(ak_bpe *m, uint32_t n, const uint8_t *tok_bytes, const uint64_t *tok_offs, const uint8_t *special);
int ak_bpe_decode(const ak_bpe *m, ak_ws *ws, const uint32_t *ids, const uint64_t *id_offs, uint64_t n, uint8_t *out,
                  uint64_t cap, uint64_t *out_offs, void *stream);
int ak_spm_decode(const ak_spm *m, ak_ws *ws, const uint32_t *ids, const uint64_t *id_offs, uint64_t n, uint8_t *out,
                  uint64_t cap, uint64_t *out_offs, void *stream);

/* Always-sufficient output capacities (elements) for n rows of total_bytes input bytes.
 * ak_bpe_encode_cap holds for flags 2 / 3; with clean_hinglish=False (flags 0 / 1) NFKC can
 * expand a char (U+FDFA: 3 bytes -> 18 code points): AK_BPE_NFKC_EXPANSION * total_bytes + 2n + 16. */
#define AK_BPE_NFKC_EXPANSION 6
uint64_t ak_normalize_cap(uint64_t n, uint64_t total_bytes);
uint64_t ak_segment_cap(uint64_t n, uint64_t total_bytes);
uint64_t ak_bpe_encode_cap(uint64_t n, uint64_t total_bytes);
uint64_t ak_spm_encode_cap(uint64_t n, uint64_t total_bytes);

#ifdef __cplusplus
}
#endif
#endif /* AKSHAR_H */
