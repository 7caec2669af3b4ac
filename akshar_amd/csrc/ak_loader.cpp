// ak_loader.cpp — model files -> the arrays ak_bpe_create / ak_spm_create take, inside the library,
// so a caller over the C-ABI (cgo, JNI, N-API, ...) needs no tokenizer.json or protobuf parser of
// its own (SURVEY.md §8(b) ak_model_load). Host code only; the same acceptance rules as the Python
// readers (akshar_amd/models.py), which the tests check array for array (tests/test_loader.py).
//
// Replaces the reference's _load_model backends (/root/reference/src/akshar/tokenizer.py:73-102):
//   BPE            Tokenizer.from_file(path)               :96-97  (the model cli.py:276-299 trains)
//   sentencepiece  SentencePieceProcessor().Load(path)    :88-90  (the model cli.py:232-248 trains)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "akshar.h"

namespace ak {
int set_error(int code, const char *msg);  // ak_engine.hip: sets ak_last_error()
int model_kind(const void *h);             // ak_engine.hip: 1 ak_bpe, 2 ak_spm, 0 neither
}  // namespace ak
static int ak_internal_model_kind(const void *h) { return ak::model_kind(h); }
static int ak_internal_fail(int code, const char *msg) { return ak::set_error(code, msg); }

namespace {

// ------------------------------------------------------------------------------------------
// a small JSON DOM (RFC 8259): objects keep their member order, strings are UTF-8

struct JVal {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double num = 0;
    std::string str;
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;
    const JVal *get(const char *key) const {
        if (kind != OBJ) return nullptr;
        for (const auto &kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    bool is_null_or_missing() const { return kind == NUL; }
};

struct JParser {
    const char *p, *e;
    std::string err;
    void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p; }
    bool fail(const char *m) { if (err.empty()) err = m; return false; }
    static void put_utf8(std::string &s, uint32_t c) {
        if (c < 0x80) s += (char)c;
        else if (c < 0x800) { s += (char)(0xC0 | (c >> 6)); s += (char)(0x80 | (c & 63)); }
        else if (c < 0x10000) { s += (char)(0xE0 | (c >> 12)); s += (char)(0x80 | ((c >> 6) & 63)); s += (char)(0x80 | (c & 63)); }
        else { s += (char)(0xF0 | (c >> 18)); s += (char)(0x80 | ((c >> 12) & 63)); s += (char)(0x80 | ((c >> 6) & 63)); s += (char)(0x80 | (c & 63)); }
    }
    bool hex4(uint32_t &v) {
        if (e - p < 4) return fail("bad \\u escape");
        v = 0;
        for (int i = 0; i < 4; ++i) {
            const char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else return fail("bad \\u escape");
        }
        return true;
    }
    bool string(std::string &s) {
        if (p >= e || *p != '"') return fail("expected a string");
        ++p;
        while (p < e && *p != '"') {
            if (*p != '\\') { s += *p++; continue; }
            if (++p >= e) return fail("bad escape");
            const char c = *p++;
            switch (c) {
                case '"': s += '"'; break;
                case '\\': s += '\\'; break;
                case '/': s += '/'; break;
                case 'b': s += '\b'; break;
                case 'f': s += '\f'; break;
                case 'n': s += '\n'; break;
                case 'r': s += '\r'; break;
                case 't': s += '\t'; break;
                case 'u': {
                    uint32_t v;
                    if (!hex4(v)) return false;
                    if (v >= 0xD800 && v < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                        const char *save = p;
                        p += 2;
                        uint32_t lo;
                        if (!hex4(lo)) return false;
                        if (lo >= 0xDC00 && lo < 0xE000) v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
                        else p = save;  // a lone high surrogate, kept as is (Python's json does the same)
                    }
                    put_utf8(s, v);
                    break;
                }
                default: return fail("bad escape");
            }
        }
        if (p >= e) return fail("unterminated string");
        ++p;
        return true;
    }
    bool value(JVal &v, int depth) {
        if (depth > 64) return fail("nesting too deep");
        ws();
        if (p >= e) return fail("unexpected end");
        const char c = *p;
        if (c == '{') {
            v.kind = JVal::OBJ;
            ++p;
            ws();
            if (p < e && *p == '}') { ++p; return true; }
            for (;;) {
                ws();
                std::string k;
                if (!string(k)) return false;
                ws();
                if (p >= e || *p != ':') return fail("expected ':'");
                ++p;
                v.obj.emplace_back(std::move(k), JVal());
                if (!value(v.obj.back().second, depth + 1)) return false;
                ws();
                if (p < e && *p == ',') { ++p; continue; }
                if (p < e && *p == '}') { ++p; return true; }
                return fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.kind = JVal::ARR;
            ++p;
            ws();
            if (p < e && *p == ']') { ++p; return true; }
            for (;;) {
                v.arr.emplace_back();
                if (!value(v.arr.back(), depth + 1)) return false;
                ws();
                if (p < e && *p == ',') { ++p; continue; }
                if (p < e && *p == ']') { ++p; return true; }
                return fail("expected ',' or ']'");
            }
        }
        if (c == '"') { v.kind = JVal::STR; return string(v.str); }
        if (e - p >= 4 && !strncmp(p, "null", 4)) { p += 4; v.kind = JVal::NUL; return true; }
        if (e - p >= 4 && !strncmp(p, "true", 4)) { p += 4; v.kind = JVal::BOOL; v.b = true; return true; }
        if (e - p >= 5 && !strncmp(p, "false", 5)) { p += 5; v.kind = JVal::BOOL; v.b = false; return true; }
        if (c == '-' || (c >= '0' && c <= '9')) {
            std::string t;
            while (p < e && (strchr("+-.eE", *p) || (*p >= '0' && *p <= '9'))) t += *p++;
            char *end = nullptr;
            v.kind = JVal::NUM;
            v.num = strtod(t.c_str(), &end);
            if (!end || *end) return fail("bad number");
            return true;
        }
        return fail("unexpected character");
    }
};

bool read_file(const char *path, std::string &out) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, k);
    fclose(f);
    return true;
}

int fail(int code, const std::string &m) { return ak_internal_fail(code, m.c_str()); }

uint32_t first_cp(const std::string &s, int *nchars) {  // the first code point + the count of code points
    uint32_t cp = 0;
    int n = 0;
    for (size_t i = 0; i < s.size();) {
        const unsigned char c = (unsigned char)s[i];
        const int l = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
        if (n == 0) {
            cp = l == 1 ? c : l == 2 ? (c & 31u) : l == 3 ? (c & 15u) : (c & 7u);
            for (int k = 1; k < l && i + k < s.size(); ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 63u);
        }
        ++n;
        i += (size_t)l;
    }
    *nchars = n;
    return cp;
}

uint64_t fnv_add(uint64_t h, const void *p, size_t n) {
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ULL; }
    return h;
}

// ------------------------------------------------------------------------------------------
// HF tokenizer.json (BPE) -> the arrays of akshar_amd/models.py BPEModel

struct BpeArrays {
    std::vector<uint32_t> single_cp, single_id, merges;  // merges: {left, right, new} per rank
    uint32_t bos = 0, eos = 0;
    std::vector<uint32_t> added_cps, added_offs{0}, added_ids;
    uint32_t vocab_size = 0;
    std::vector<uint8_t> tok_bytes, special;
    std::vector<uint64_t> tok_offs{0};
};

// a token id as the model file states it: a JSON number that is a whole number in [0, 2^24)
// (anything else would wrap the u32 ids or size a decode table by a garbage value)
static bool json_id(const JVal *v, uint32_t &out) {
    if (!v || v->kind != JVal::NUM) return false;
    const double x = v->num;
    if (!(x >= 0.0) || x >= 16777216.0 || x != (double)(uint32_t)x) return false;
    out = (uint32_t)x;
    return true;
}

int parse_bpe(const char *path, BpeArrays &A) {
    std::string text;
    if (!read_file(path, text)) return fail(AK_ERR_ARG, std::string("cannot read ") + path);
    JParser P{text.data(), text.data() + text.size(), ""};
    JVal root;
    if (!P.value(root, 0)) return fail(AK_ERR_ARG, "tokenizer.json: " + P.err);
    const JVal *m = root.get("model");
    const JVal *ty = m ? m->get("type") : nullptr;
    if (!ty || ty->kind != JVal::STR || ty->str != "BPE") return fail(AK_ERR_UNSUPPORTED, "only BPE tokenizer.json models are supported");
    for (const char *k : {"dropout", "unk_token", "continuing_subword_prefix", "end_of_word_suffix"}) {
        const JVal *v = m->get(k);
        if (v && !v->is_null_or_missing() && !(v->kind == JVal::NUM && v->num == 0.0 && !strcmp(k, "dropout")))
            return fail(AK_ERR_UNSUPPORTED, std::string("BPE option ") + k + " not supported");
    }
    for (const char *k : {"byte_fallback", "ignore_merges"}) {
        const JVal *v = m->get(k);
        if (v && !(v->kind == JVal::BOOL && !v->b) && !v->is_null_or_missing())
            return fail(AK_ERR_UNSUPPORTED, std::string("BPE option ") + k + " not supported");
    }
    const JVal *nz = root.get("normalizer");
    const JVal *nt = nz ? nz->get("type") : nullptr;
    if (!nt || nt->str != "NFKC") return fail(AK_ERR_UNSUPPORTED, "BPE normalizer must be NFKC (cli.py:278)");
    const JVal *pt = root.get("pre_tokenizer");
    const JVal *ptt = pt ? pt->get("type") : nullptr;
    if (!ptt || ptt->str != "Whitespace") return fail(AK_ERR_UNSUPPORTED, "BPE pre_tokenizer must be Whitespace (cli.py:279)");
    const JVal *voc = m->get("vocab");
    if (!voc || voc->kind != JVal::OBJ) return fail(AK_ERR_ARG, "tokenizer.json: model.vocab missing");
    std::map<std::string, uint32_t> vocab;
    std::vector<std::pair<uint32_t, uint32_t>> singles;
    for (const auto &kv : voc->obj) {
        uint32_t id = 0;
        if (!json_id(&kv.second, id)) return fail(AK_ERR_ARG, "tokenizer.json: vocab id of " + kv.first + " is not an integer in [0, 2^24)");
        vocab[kv.first] = id;
        int nch = 0;
        const uint32_t cp = first_cp(kv.first, &nch);
        if (nch == 1) singles.push_back({cp, id});
    }
    const JVal *added = root.get("added_tokens");
    std::vector<std::pair<std::string, uint32_t>> added_list;
    std::vector<uint32_t> special_ids;
    if (added && added->kind == JVal::ARR) {
        for (const JVal &a : added->arr) {
            const JVal *c = a.get("content"), *i = a.get("id");
            uint32_t aid = 0;
            if (!c || c->kind != JVal::STR || !json_id(i, aid))
                return fail(AK_ERR_ARG, "tokenizer.json: added token without a string content / an integer id in [0, 2^24)");
            vocab.emplace(c->str, aid);  // setdefault
            for (const char *k : {"single_word", "lstrip", "rstrip", "normalized"}) {
                const JVal *f = a.get(k);
                if (f && f->kind == JVal::BOOL && f->b)
                    return fail(AK_ERR_UNSUPPORTED, "added token " + c->str + " with " + k + "=True not supported");
            }
            added_list.push_back({c->str, aid});
            const JVal *sp = a.get("special");
            if (sp && sp->kind == JVal::BOOL && sp->b) special_ids.push_back(aid);
        }
    }
    std::sort(singles.begin(), singles.end());
    for (auto &s : singles) { A.single_cp.push_back(s.first); A.single_id.push_back(s.second); }
    const JVal *mg = m->get("merges");
    if (mg && mg->kind == JVal::ARR) {
        for (const JVal &x : mg->arr) {
            std::string a, b;
            if (x.kind == JVal::STR) {
                const size_t sp = x.str.find(' ');
                if (sp == std::string::npos) return fail(AK_ERR_ARG, "tokenizer.json: bad merge " + x.str);
                a = x.str.substr(0, sp);
                b = x.str.substr(sp + 1);
            } else if (x.kind == JVal::ARR && x.arr.size() == 2) {
                a = x.arr[0].str;
                b = x.arr[1].str;
            } else {
                return fail(AK_ERR_ARG, "tokenizer.json: bad merge entry");
            }
            auto ia = vocab.find(a), ib = vocab.find(b), iab = vocab.find(a + b);
            if (ia == vocab.end() || ib == vocab.end() || iab == vocab.end())
                return fail(AK_ERR_ARG, "tokenizer.json: merge of tokens outside the vocabulary");
            A.merges.insert(A.merges.end(), {ia->second, ib->second, iab->second});
        }
    }
    const JVal *pp = root.get("post_processor");
    const JVal *ppt = pp ? pp->get("type") : nullptr;
    const JVal *single = (ppt && ppt->str == "TemplateProcessing") ? pp->get("single") : nullptr;
    if (!single || single->kind != JVal::ARR || single->arr.size() != 3)
        return fail(AK_ERR_UNSUPPORTED, "BPE post_processor must be the <s> $A </s> template (cli.py:286-293)");
    const JVal *s0 = single->arr[0].get("SpecialToken"), *s1 = single->arr[1].get("Sequence"),
               *s2 = single->arr[2].get("SpecialToken");
    if (!s0 || !s1 || !s2 || single->arr[1].get("SpecialToken")) return fail(AK_ERR_UNSUPPORTED, "unsupported template");
    const JVal *n0 = s0->get("id"), *n2 = s2->get("id");
    if (!n0 || n0->kind != JVal::STR || !n2 || n2->kind != JVal::STR)
        return fail(AK_ERR_UNSUPPORTED, "template SpecialToken without a string id");
    const JVal *st = pp->get("special_tokens");
    const JVal *b0 = st ? st->get(n0->str.c_str()) : nullptr;
    const JVal *b2 = st ? st->get(n2->str.c_str()) : nullptr;
    const JVal *i0 = b0 ? b0->get("ids") : nullptr, *i2 = b2 ? b2->get("ids") : nullptr;
    if (!i0 || !i2 || i0->kind != JVal::ARR || i2->kind != JVal::ARR || i0->arr.empty() || i2->arr.empty())
        return fail(AK_ERR_UNSUPPORTED, "template special tokens without ids");
    if (!json_id(&i0->arr[0], A.bos) || !json_id(&i2->arr[0], A.eos))
        return fail(AK_ERR_ARG, "tokenizer.json: template special token id is not an integer in [0, 2^24)");
    for (auto &a : added_list) {
        uint32_t cnt = 0;
        for (size_t i = 0; i < a.first.size();) {
            const unsigned char c = (unsigned char)a.first[i];
            const int l = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
            int dummy;
            A.added_cps.push_back(first_cp(a.first.substr(i, (size_t)l), &dummy));
            i += (size_t)l;
            ++cnt;
        }
        A.added_offs.push_back(A.added_offs.back() + cnt);
        A.added_ids.push_back(a.second);
    }
    // decode vocabulary: ids 0 .. max id, missing ids empty and flagged like special tokens
    std::map<uint32_t, std::string> id_to_tok;
    for (auto &kv : vocab) id_to_tok[kv.second] = kv.first;  // (ids are unique in a trained model)
    A.vocab_size = id_to_tok.empty() ? 0 : id_to_tok.rbegin()->first + 1;
    for (uint32_t i = 0; i < A.vocab_size; ++i) {
        auto it = id_to_tok.find(i);
        const bool sp = it == id_to_tok.end() || std::find(special_ids.begin(), special_ids.end(), i) != special_ids.end();
        if (it != id_to_tok.end()) A.tok_bytes.insert(A.tok_bytes.end(), it->second.begin(), it->second.end());
        A.tok_offs.push_back(A.tok_bytes.size());
        A.special.push_back(sp ? 1 : 0);
    }
    return AK_OK;
}

// ------------------------------------------------------------------------------------------
// SentencePiece ModelProto (sentencepiece_model.proto wire format) -> akshar_amd/models.py SPMModel

struct SpmArrays {
    std::vector<uint8_t> piece_bytes;
    std::vector<uint64_t> piece_offs{0};
    std::vector<float> scores;
    std::vector<uint8_t> types;
    int32_t unk_id = -1;
    int32_t byte_ids[256];
};

struct PbField { uint32_t fn, wt; uint64_t v; const uint8_t *p; size_t n; };

bool pb_varint(const uint8_t *&p, const uint8_t *e, uint64_t &x) {
    x = 0;
    for (int s = 0; s < 64 && p < e; s += 7) {
        const uint8_t b = *p++;
        x |= (uint64_t)(b & 0x7F) << s;
        if (b < 0x80) return true;
    }
    return false;
}

bool pb_fields(const uint8_t *p, const uint8_t *e, std::vector<PbField> &out) {
    while (p < e) {
        uint64_t key;
        if (!pb_varint(p, e, key)) return false;
        PbField f{(uint32_t)(key >> 3), (uint32_t)(key & 7), 0, nullptr, 0};
        if (f.wt == 0) { if (!pb_varint(p, e, f.v)) return false; }
        else if (f.wt == 1) { if (e - p < 8) return false; f.p = p; f.n = 8; p += 8; }
        else if (f.wt == 2) {
            uint64_t ln;
            if (!pb_varint(p, e, ln) || (uint64_t)(e - p) < ln) return false;
            f.p = p; f.n = (size_t)ln; p += ln;
        } else if (f.wt == 5) { if (e - p < 4) return false; f.p = p; f.n = 4; p += 4; }
        else return false;
        out.push_back(f);
    }
    return true;
}

int parse_spm(const char *path, SpmArrays &A) {
    std::string buf;
    if (!read_file(path, buf)) return fail(AK_ERR_ARG, std::string("cannot read ") + path);
    const uint8_t *b = (const uint8_t *)buf.data();
    std::vector<PbField> top;
    if (!pb_fields(b, b + buf.size(), top)) return fail(AK_ERR_ARG, "bad SentencePiece model protobuf");
    const PbField *trainer = nullptr, *normalizer = nullptr;
    for (const PbField &f : top) {
        if (f.fn == 1 && f.wt == 2) {
            std::vector<PbField> pf;
            if (!pb_fields(f.p, f.p + f.n, pf)) return fail(AK_ERR_ARG, "bad SentencePiece piece");
            std::string piece;
            float score = 0.0f;
            uint8_t type = 1;
            for (const PbField &g : pf) {
                if (g.fn == 1 && g.wt == 2) piece.assign((const char *)g.p, g.n);
                else if (g.fn == 2 && g.wt == 5) memcpy(&score, g.p, 4);
                else if (g.fn == 3 && g.wt == 0) type = (uint8_t)g.v;
            }
            A.piece_bytes.insert(A.piece_bytes.end(), piece.begin(), piece.end());
            A.piece_offs.push_back(A.piece_bytes.size());
            A.scores.push_back(score);
            A.types.push_back(type);
        } else if (f.fn == 2 && f.wt == 2) {
            trainer = &f;
        } else if (f.fn == 3 && f.wt == 2) {
            normalizer = &f;
        }
    }
    std::map<uint32_t, uint64_t> tr, nm;
    std::vector<PbField> tf, nf;
    if (trainer && !pb_fields(trainer->p, trainer->p + trainer->n, tf)) return fail(AK_ERR_ARG, "bad trainer_spec");
    if (normalizer && !pb_fields(normalizer->p, normalizer->p + normalizer->n, nf)) return fail(AK_ERR_ARG, "bad normalizer_spec");
    for (const PbField &f : tf) if (f.wt == 0) tr[f.fn] = f.v;
    bool charsmap = false;
    for (const PbField &f : nf) {
        if (f.wt == 0) nm[f.fn] = f.v;
        if (f.fn == 2 && f.wt == 2 && f.n > 0) charsmap = true;
    }
    auto get = [](const std::map<uint32_t, uint64_t> &m, uint32_t k, uint64_t d) { auto it = m.find(k); return it == m.end() ? d : it->second; };
    if (get(tr, 3, 1) != 1) return fail(AK_ERR_UNSUPPORTED, "only SentencePiece unigram models are supported (cli.py:240)");
    if (get(tr, 24, 0)) return fail(AK_ERR_UNSUPPORTED, "treat_whitespace_as_suffix is not supported");
    if (charsmap) return fail(AK_ERR_UNSUPPORTED, "only the identity normalizer (empty charsmap) is supported (cli.py:243)");
    if (!get(nm, 3, 1) || !get(nm, 4, 1) || !get(nm, 5, 1))
        return fail(AK_ERR_UNSUPPORTED, "normalizer flags other than the defaults are not supported");
    if (!get(tr, 35, 0)) return fail(AK_ERR_UNSUPPORTED, "only byte_fallback models are supported (cli.py:244)");
    int n_unk = 0;
    for (int i = 0; i < 256; ++i) A.byte_ids[i] = -1;
    for (size_t i = 0; i < A.types.size(); ++i) {
        if (A.types[i] == 2) { A.unk_id = (int32_t)i; ++n_unk; }
        const uint64_t o = A.piece_offs[i], l = A.piece_offs[i + 1] - o;
        const char *s = (const char *)A.piece_bytes.data() + o;
        if (A.types[i] == 6 && l == 6 && !strncmp(s, "<0x", 3) && s[5] == '>') {
            char hx[3] = {s[3], s[4], 0};
            A.byte_ids[strtol(hx, nullptr, 16) & 255] = (int32_t)i;
        }
    }
    if (n_unk != 1) return fail(AK_ERR_UNSUPPORTED, "model must have exactly one <unk> piece");
    for (int i = 0; i < 256; ++i)
        if (A.byte_ids[i] < 0) return fail(AK_ERR_UNSUPPORTED, "byte_fallback model without all 256 byte pieces");
    return AK_OK;
}

bool is_bpe(const char *t) { return t && (!strcmp(t, "bpe") || !strcmp(t, "BPE")); }
bool is_spm(const char *t) { return t && (!strcmp(t, "sentencepiece") || !strcmp(t, "spm") || !strcmp(t, "unigram")); }

}  // namespace

extern "C" int ak_bpe_load(const char *path, ak_bpe **out) {
    if (!path || !out) return ak_internal_fail(AK_ERR_ARG, "ak_bpe_load: null argument");
    BpeArrays A;
    int rc = parse_bpe(path, A);
    if (rc) return rc;
    ak_bpe *m = nullptr;
    rc = ak_bpe_create((uint32_t)A.single_cp.size(), A.single_cp.data(), A.single_id.data(), (uint32_t)(A.merges.size() / 3),
                       A.merges.data(), A.bos, A.eos, &m);
    if (rc) return rc;
    rc = ak_bpe_set_added(m, (uint32_t)A.added_ids.size(), A.added_cps.data(), A.added_offs.data(), A.added_ids.data());
    if (!rc) {
        const uint8_t z = 0;
        rc = ak_bpe_set_vocab(m, A.vocab_size, A.tok_bytes.empty() ? &z : A.tok_bytes.data(), A.tok_offs.data(), A.special.data());
    }
    if (rc) { ak_bpe_free(m); return rc; }
    *out = m;
    return AK_OK;
}

extern "C" int ak_spm_load(const char *path, ak_spm **out) {
    if (!path || !out) return ak_internal_fail(AK_ERR_ARG, "ak_spm_load: null argument");
    SpmArrays A;
    int rc = parse_spm(path, A);
    if (rc) return rc;
    return ak_spm_create((uint32_t)A.types.size(), A.piece_bytes.data(), A.piece_offs.data(), A.scores.data(),
                         A.types.data(), A.unk_id, A.byte_ids, out);
}

extern "C" int ak_model_load(const char *path, const char *model_type, void **out) {
    if (is_bpe(model_type)) return ak_bpe_load(path, (ak_bpe **)out);
    if (is_spm(model_type)) return ak_spm_load(path, (ak_spm **)out);
    return ak_internal_fail(AK_ERR_ARG, "ak_model_load: model_type must be \"bpe\" or \"sentencepiece\"");
}

// The handle carries its kind (ak_engine.hip model_kind), so the type string only has to agree:
// a mismatched or unknown model_type still frees the handle by its own kind and records an error
// (ak_last_error); a handle that is neither kind is left alone and recorded.
extern "C" void ak_model_free(void *h, const char *model_type) {
    if (!h) return;
    const int kind = ak_internal_model_kind(h);
    if (kind == 1) ak_bpe_free((ak_bpe *)h);
    else if (kind == 2) ak_spm_free((ak_spm *)h);
    if (kind == 0) (void)ak_internal_fail(AK_ERR_ARG, "ak_model_free: not a model handle (left alone)");
    else if (!(kind == 1 ? is_bpe(model_type) : is_spm(model_type)))
        (void)ak_internal_fail(AK_ERR_ARG, "ak_model_free: model_type does not match the handle (freed by its kind)");
}

extern "C" int ak_model_info(const char *path, const char *model_type, uint64_t info[8]) {
    if (!path || !info) return ak_internal_fail(AK_ERR_ARG, "ak_model_info: null argument");
    memset(info, 0, 8 * sizeof(uint64_t));
    uint64_t h = 1469598103934665603ULL;
    if (is_bpe(model_type)) {
        BpeArrays A;
        int rc = parse_bpe(path, A);
        if (rc) return rc;
        h = fnv_add(h, A.single_cp.data(), A.single_cp.size() * 4);
        h = fnv_add(h, A.single_id.data(), A.single_id.size() * 4);
        h = fnv_add(h, A.merges.data(), A.merges.size() * 4);
        h = fnv_add(h, A.added_cps.data(), A.added_cps.size() * 4);
        h = fnv_add(h, A.added_offs.data(), A.added_offs.size() * 4);
        h = fnv_add(h, A.added_ids.data(), A.added_ids.size() * 4);
        h = fnv_add(h, A.tok_bytes.data(), A.tok_bytes.size());
        h = fnv_add(h, A.tok_offs.data(), A.tok_offs.size() * 8);
        h = fnv_add(h, A.special.data(), A.special.size());
        const uint64_t v[8] = {A.vocab_size, A.single_cp.size(), A.merges.size() / 3, A.bos, A.eos, A.added_ids.size(), 0, h};
        memcpy(info, v, sizeof(v));
        return AK_OK;
    }
    if (is_spm(model_type)) {
        SpmArrays A;
        int rc = parse_spm(path, A);
        if (rc) return rc;
        h = fnv_add(h, A.piece_bytes.data(), A.piece_bytes.size());
        h = fnv_add(h, A.piece_offs.data(), A.piece_offs.size() * 8);
        h = fnv_add(h, A.scores.data(), A.scores.size() * 4);
        h = fnv_add(h, A.types.data(), A.types.size());
        h = fnv_add(h, A.byte_ids, sizeof(A.byte_ids));
        const uint64_t v[8] = {A.types.size(), (uint64_t)A.unk_id, 0, 0, 0, 0, 0, h};
        memcpy(info, v, sizeof(v));
        return AK_OK;
    }
    return ak_internal_fail(AK_ERR_ARG, "ak_model_info: model_type must be \"bpe\" or \"sentencepiece\"");
}
