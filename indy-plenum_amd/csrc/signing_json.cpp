// pv_signing_serialize_json: signing serialization of received JSON requests, in C++, many threads
// (SURVEY.md §8f-3).
//
// Reference semantics, applied to json.loads(text) — the dict ZStack.deserializeMsg produces from the
// wire bytes (stp_zmq/zstack.py:881-885; `msg.decode()` is strict UTF-8):
//   SigningSerializer.serialize (common/serializers/signing_serializer.py:35-92) via
//   serialize_msg_for_signing (common/serializers/serialization.py:27-36): str -> itself, int ->
//   str(int), True/False -> "True"/"False", None -> "", list -> items joined by ",", dict -> keys
//   sorted, "k:v" joined by "|" (nested keys are NOT prefixed: the INDY-1469 ambiguity is kept).
// Modes:
//   PV_SER_DICT     serialize(obj)
//   PV_SER_AUTHN    serialize(obj minus top-level {signature, signatures, fees})
//                   (CoreAuthMixin.authenticate, plenum/server/client_authn.py:198,232)
//   PV_SER_REQUEST  serialize(Request(**obj).as_dict minus those keys) — what Node.verifySignature
//                   verifies (plenum/server/node.py:2636-2650, plenum/common/request.py:53-74) — and
//                   digest = sha256(serialize(signingState())) (request.py:86-121), the cache key.
// Anything this serializer does not reproduce bit-for-bit is reported, never approximated: floats
// (repr() rounding), NaN/Infinity, lone UTF-16 surrogates (encode('utf-8') raises), nesting deeper
// than 512, integers longer than Python's 4,300-digit str() limit and request-mode digests whose
// Python evaluation raises get status PV_SER_DEFER, and the caller serializes those in Python.
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <string_view>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/plenum_verify.h"

int pv_fail(int code, const std::string& msg);  // pv_engine.hip

namespace {

// ------------------------------------------------------------------------- SHA-256 (FIPS 180-4)
const uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void sha256_compress(uint32_t st[8], const uint8_t* blk) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 | (uint32_t)blk[4 * i + 2] << 8 |
               (uint32_t)blk[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t v[8];
    memcpy(v, st, sizeof v);
    for (int i = 0; i < 64; i++) {
        const uint32_t t1 = v[7] + (rotr(v[4], 6) ^ rotr(v[4], 11) ^ rotr(v[4], 25)) + ((v[4] & v[5]) ^ (~v[4] & v[6])) +
                            kSha256K[i] + w[i];
        const uint32_t t2 = (rotr(v[0], 2) ^ rotr(v[0], 13) ^ rotr(v[0], 22)) +
                            ((v[0] & v[1]) ^ (v[0] & v[2]) ^ (v[1] & v[2]));
        memmove(v + 1, v, 7 * sizeof(uint32_t));
        v[4] += t1;
        v[0] = t1 + t2;
    }
    for (int i = 0; i < 8; i++) st[i] += v[i];
}

// The same compression on the x86 SHA extensions (every request digest of the wire path hashes
// ~7 blocks; this is ~8x the scalar rate). State kept as (ABEF, CDGH), the layout sha256rnds2 uses;
// four rounds per 128-bit message group, the schedule W[t] = s1(W[t-2]) + W[t-7] + s0(W[t-15]) +
// W[t-16] as sha256msg1 (W[t-16] + s0), an alignr for W[t-7], sha256msg2 (s1).
__attribute__((target("sha,sse4.1,ssse3"))) void sha256_compress_ni(uint32_t st[8], const uint8_t* data, size_t nblk) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i t = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(st)), 0xB1);     // C D A B
    __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(st + 4)), 0x1B);  // E F G H
    __m128i s0 = _mm_alignr_epi8(t, s1, 8);  // A B E F
    s1 = _mm_blend_epi16(s1, t, 0xF0);       // C D G H
    for (; nblk; nblk--, data += 64) {
        const __m128i abef = s0, cdgh = s1;
        __m128i w[4];
#pragma GCC unroll 16
        for (int g = 0; g < 16; g++) {
            __m128i m;
            if (g < 4) {
                m = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 16 * g)), bswap);
            } else {
                m = _mm_sha256msg1_epu32(w[g & 3], w[(g + 1) & 3]);
                m = _mm_add_epi32(m, _mm_alignr_epi8(w[(g + 3) & 3], w[(g + 2) & 3], 4));
                m = _mm_sha256msg2_epu32(m, w[(g + 3) & 3]);
            }
            w[g & 3] = m;
            __m128i k = _mm_add_epi32(m, _mm_loadu_si128(reinterpret_cast<const __m128i*>(kSha256K + 4 * g)));
            s1 = _mm_sha256rnds2_epu32(s1, s0, k);
            s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(k, 0x0E));
        }
        s0 = _mm_add_epi32(s0, abef);
        s1 = _mm_add_epi32(s1, cdgh);
    }
    t = _mm_shuffle_epi32(s0, 0x1B);   // F E B A
    s1 = _mm_shuffle_epi32(s1, 0xB1);  // D C H G
    _mm_storeu_si128(reinterpret_cast<__m128i*>(st), _mm_blend_epi16(t, s1, 0xF0));     // D C B A
    _mm_storeu_si128(reinterpret_cast<__m128i*>(st + 4), _mm_alignr_epi8(s1, t, 8));     // H G F E
}

const bool kShaNi = __builtin_cpu_supports("sha");

void sha256_blocks(uint32_t st[8], const uint8_t* data, size_t nblk) {
    if (kShaNi) return sha256_compress_ni(st, data, nblk);
    for (; nblk; nblk--, data += 64) sha256_compress(st, data);
}

void sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    const size_t full = len / 64;
    sha256_blocks(st, data, full);
    const size_t i = 64 * full;
    uint8_t tail[128] = {0};
    const size_t rem = len - i;
    memcpy(tail, data + i, rem);
    tail[rem] = 0x80;
    const size_t tl = rem + 9 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)len * 8;
    for (int k = 0; k < 8; k++) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
    sha256_blocks(st, tail, tl / 64);
    for (int k = 0; k < 8; k++) {
        out[4 * k] = (uint8_t)(st[k] >> 24);
        out[4 * k + 1] = (uint8_t)(st[k] >> 16);
        out[4 * k + 2] = (uint8_t)(st[k] >> 8);
        out[4 * k + 3] = (uint8_t)st[k];
    }
}

// ------------------------------------------------------------------- JSON as Python's json.loads
enum Kind : uint8_t { J_NULL, J_FALSE, J_TRUE, J_INT, J_STR, J_ARR, J_OBJ };

// J_INT / J_STR: bytes text[a, b) (decoded UTF-8 / canonical decimal); J_ARR: element node ids
// kids[a, b); J_OBJ: kids[a, b) holds (key node, value node) pairs in document order.
struct JNode {
    Kind k;
    uint32_t a, b;
};

constexpr uint32_t kBad = 0xFFFFFFFFu;
constexpr int kMaxDepth = 512;
constexpr size_t kMaxIntDigits = 4300;  // CPython int <-> str conversion limit (3.10.7+)

struct Doc {
    std::string text;
    std::vector<JNode> nodes;
    std::vector<uint32_t> kids;
    std::vector<uint32_t> scratch;
    void clear() {
        text.clear();
        nodes.clear();
        kids.clear();
        scratch.clear();
    }
    uint32_t add(Kind k, uint32_t a = 0, uint32_t b = 0) {
        nodes.push_back(JNode{k, a, b});
        return (uint32_t)nodes.size() - 1;
    }
    uint32_t add_text(Kind k, const char* s, size_t n) {
        const uint32_t a = (uint32_t)text.size();
        text.append(s, n);
        return add(k, a, (uint32_t)text.size());
    }
    bool key_eq(uint32_t node, const char* s, size_t n) const {
        const JNode& x = nodes[node];
        return x.b - x.a == n && memcmp(text.data() + x.a, s, n) == 0;
    }
    int key_cmp(uint32_t p, uint32_t q) const {
        const JNode &x = nodes[p], &y = nodes[q];
        const size_t lx = x.b - x.a, ly = y.b - y.a;
        const int c = memcmp(text.data() + x.a, text.data() + y.a, std::min(lx, ly));
        return c ? c : (lx < ly ? -1 : (lx > ly ? 1 : 0));
    }
    bool truthy(uint32_t node) const {  // Python truth value of the decoded object
        const JNode& x = nodes[node];
        switch (x.k) {
            case J_NULL:
            case J_FALSE:
                return false;
            case J_TRUE:
                return true;
            case J_INT:
                return !(x.b - x.a == 1 && text[x.a] == '0');
            default:
                return x.b > x.a;
        }
    }
};

// strict UTF-8 (bytes.decode()): no overlong forms, no surrogates, nothing above U+10FFFF
bool utf8_valid(const uint8_t* s, size_t n) {
    size_t i = 0;
    while (i < n) {
        if (i + 16 <= n && !_mm_movemask_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i)))) {
            i += 16;  // 16 ASCII bytes
            continue;
        }
        const uint8_t c = s[i];
        if (c < 0x80) {
            i++;
            continue;
        }
        size_t len;
        uint32_t cp;
        if (c >= 0xC2 && c <= 0xDF) {
            len = 2;
            cp = c & 0x1F;
        } else if (c >= 0xE0 && c <= 0xEF) {
            len = 3;
            cp = c & 0x0F;
        } else if (c >= 0xF0 && c <= 0xF4) {
            len = 4;
            cp = c & 0x07;
        } else {
            return false;
        }
        if (i + len > n) return false;
        for (size_t k = 1; k < len; k++) {
            if ((s[i + k] & 0xC0) != 0x80) return false;
            cp = cp << 6 | (s[i + k] & 0x3F);
        }
        if (len == 3 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) return false;
        if (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) return false;
        i += len;
    }
    return true;
}

void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) {
        o += (char)cp;
    } else if (cp < 0x800) {
        o += (char)(0xC0 | cp >> 6);
        o += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
        o += (char)(0xE0 | cp >> 12);
        o += (char)(0x80 | ((cp >> 6) & 0x3F));
        o += (char)(0x80 | (cp & 0x3F));
    } else {
        o += (char)(0xF0 | cp >> 18);
        o += (char)(0x80 | ((cp >> 12) & 0x3F));
        o += (char)(0x80 | ((cp >> 6) & 0x3F));
        o += (char)(0x80 | (cp & 0x3F));
    }
}

inline bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }

// The grammar of CPython's json scanner (Lib/json/decoder.py + Modules/_json.c, strict=True).
struct Parser {
    const uint8_t* p;
    const uint8_t* e;
    Doc& d;
    bool defer = false;  // parsed, but outside what the native serializer reproduces
    int err = PV_SER_OK;

    uint32_t fail(int s) {
        if (err == PV_SER_OK) err = s;
        return kBad;
    }
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
    }
    bool lit(const char* s, size_t n) {
        if ((size_t)(e - p) < n || memcmp(p, s, n) != 0) return false;
        p += n;
        return true;
    }
    int hex4(const uint8_t* q) const {
        if (e - q < 4) return -1;
        int v = 0;
        for (int i = 0; i < 4; i++) {
            const uint8_t c = q[i];
            int h;
            if (c >= '0' && c <= '9')
                h = c - '0';
            else if (c >= 'a' && c <= 'f')
                h = c - 'a' + 10;
            else if (c >= 'A' && c <= 'F')
                h = c - 'A' + 10;
            else
                return -1;
            v = v << 4 | h;
        }
        return v;
    }

    uint32_t str() {
        p++;  // opening quote
        const uint32_t a = (uint32_t)d.text.size();
        for (;;) {
            if (p >= e) return fail(PV_SER_INVALID);
            const uint8_t c = *p;
            if (c == '"') {
                p++;
                break;
            }
            if (c < 0x20) return fail(PV_SER_INVALID);  // strict: control characters
            if (c != '\\') {
                const uint8_t* r = p;
                // 16 bytes at a time up to the first quote, backslash or control character
                const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), ctl = _mm_set1_epi8(0x1F);
                while (e - p >= 16) {
                    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
                    const __m128i hit = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs)),
                                                     _mm_cmpeq_epi8(_mm_max_epu8(x, ctl), ctl));
                    const int m = _mm_movemask_epi8(hit);
                    if (m) {
                        p += __builtin_ctz((unsigned)m);
                        break;
                    }
                    p += 16;
                }
                while (p < e && *p != '"' && *p != '\\' && *p >= 0x20) p++;
                d.text.append(reinterpret_cast<const char*>(r), p - r);
                continue;
            }
            if (e - p < 2) return fail(PV_SER_INVALID);
            const uint8_t x = p[1];
            p += 2;
            switch (x) {
                case '"': d.text += '"'; break;
                case '\\': d.text += '\\'; break;
                case '/': d.text += '/'; break;
                case 'b': d.text += '\b'; break;
                case 'f': d.text += '\f'; break;
                case 'n': d.text += '\n'; break;
                case 'r': d.text += '\r'; break;
                case 't': d.text += '\t'; break;
                case 'u': {
                    const int u = hex4(p);
                    if (u < 0) return fail(PV_SER_INVALID);
                    p += 4;
                    if (u >= 0xD800 && u <= 0xDBFF && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                        const int u2 = hex4(p + 2);
                        if (u2 < 0) return fail(PV_SER_INVALID);
                        if (u2 >= 0xDC00 && u2 <= 0xDFFF) {
                            p += 6;
                            put_utf8(d.text, 0x10000u + ((uint32_t)(u - 0xD800) << 10) + (uint32_t)(u2 - 0xDC00));
                            break;
                        }
                    }
                    if (u >= 0xD800 && u <= 0xDFFF) defer = true;  // lone surrogate: encode() raises
                    put_utf8(d.text, (uint32_t)u);
                    break;
                }
                default:
                    return fail(PV_SER_INVALID);
            }
        }
        return d.add(J_STR, a, (uint32_t)d.text.size());
    }

    uint32_t num() {
        const uint8_t* s = p;
        const bool neg = *p == '-';
        if (neg) p++;
        if (p >= e || !is_digit(*p)) return fail(PV_SER_INVALID);
        if (*p == '0')
            p++;
        else
            while (p < e && is_digit(*p)) p++;
        const uint8_t* int_end = p;
        bool is_float = false;
        if (e - p >= 2 && *p == '.' && is_digit(p[1])) {
            p += 2;
            while (p < e && is_digit(*p)) p++;
            is_float = true;
        }
        if (p < e && (*p == 'e' || *p == 'E')) {
            const uint8_t* q = p + 1;
            if (q < e && (*q == '+' || *q == '-')) q++;
            if (q < e && is_digit(*q)) {
                p = q;
                while (p < e && is_digit(*p)) p++;
                is_float = true;
            }
        }
        const size_t digits = (size_t)(int_end - s) - (neg ? 1 : 0);
        if (is_float || digits > kMaxIntDigits) {
            defer = true;
            return d.add(J_NULL);
        }
        if (neg && digits == 1 && s[1] == '0') return d.add_text(J_INT, "0", 1);  // str(int("-0"))
        return d.add_text(J_INT, reinterpret_cast<const char*>(s), (size_t)(int_end - s));
    }

    uint32_t container(int depth, bool obj) {
        if (depth >= kMaxDepth) return fail(PV_SER_DEFER);
        p++;
        ws();
        const size_t mark = d.scratch.size();
        const uint8_t close = obj ? '}' : ']';
        if (p < e && *p == close) {
            p++;
        } else {
            for (;;) {
                if (obj) {
                    if (p >= e || *p != '"') return fail(PV_SER_INVALID);
                    const uint32_t k = str();
                    if (k == kBad) return kBad;
                    ws();
                    if (p >= e || *p != ':') return fail(PV_SER_INVALID);
                    p++;
                    ws();
                    d.scratch.push_back(k);
                }
                const uint32_t v = value(depth + 1);
                if (v == kBad) return kBad;
                d.scratch.push_back(v);
                ws();
                if (p < e && *p == ',') {
                    p++;
                    ws();
                    continue;
                }
                if (p < e && *p == close) {
                    p++;
                    break;
                }
                return fail(PV_SER_INVALID);
            }
        }
        const uint32_t a = (uint32_t)d.kids.size();
        d.kids.insert(d.kids.end(), d.scratch.begin() + mark, d.scratch.end());
        d.scratch.resize(mark);
        return d.add(obj ? J_OBJ : J_ARR, a, (uint32_t)d.kids.size());
    }

    uint32_t value(int depth) {
        if (p >= e) return fail(PV_SER_INVALID);
        switch (*p) {
            case '{':
                return container(depth, true);
            case '[':
                return container(depth, false);
            case '"':
                return str();
            case 'n':
                if (lit("null", 4)) return d.add(J_NULL);
                break;
            case 't':
                if (lit("true", 4)) return d.add(J_TRUE);
                break;
            case 'f':
                if (lit("false", 5)) return d.add(J_FALSE);
                break;
            case 'N':
                if (lit("NaN", 3)) {
                    defer = true;
                    return d.add(J_NULL);
                }
                break;
            case 'I':
                if (lit("Infinity", 8)) {
                    defer = true;
                    return d.add(J_NULL);
                }
                break;
            case '-':
                if (lit("-Infinity", 9)) {
                    defer = true;
                    return d.add(J_NULL);
                }
                return num();
            default:
                if (is_digit(*p)) return num();
        }
        return fail(PV_SER_INVALID);
    }
};

int parse(const uint8_t* s, size_t n, Doc& d, uint32_t& root) {
    d.clear();
    if (!utf8_valid(s, n)) return PV_SER_INVALID;
    Parser P{s, s + n, d};
    P.ws();
    root = P.value(0);
    if (root == kBad) return P.err;
    P.ws();
    if (P.p != P.e) return PV_SER_INVALID;  // "Extra data"
    return P.defer ? PV_SER_DEFER : PV_SER_OK;
}

// ------------------------------------------------------------------------------ serialization
void ser(const Doc& d, uint32_t x, std::string& out);

// dict: keys deduplicated (the last value wins, as in a Python dict), sorted by code point (= UTF-8
// byte order), "k:v" joined by "|"; `skip` lists top-level keys to leave out. Objects of up to 32
// members sort in a stack buffer (stable insertion sort: no allocation on the per-request path).
void ser_obj(const Doc& d, const JNode n, std::string& out, const char* const* skip, int nskip) {
    const uint32_t m = (n.b - n.a) / 2;
    uint32_t small[32];
    std::vector<uint32_t> big;
    uint32_t* order = small;
    auto less = [&](uint32_t x, uint32_t y) { return d.key_cmp(d.kids[n.a + 2 * x], d.kids[n.a + 2 * y]) < 0; };
    if (m <= 32) {
        for (uint32_t i = 0; i < m; i++) {
            uint32_t j = i;
            while (j > 0 && less(i, order[j - 1])) {
                order[j] = order[j - 1];
                j--;
            }
            order[j] = i;
        }
    } else {
        big.resize(m);
        for (uint32_t i = 0; i < m; i++) big[i] = i;
        std::stable_sort(big.begin(), big.end(), less);
        order = big.data();
    }
    bool first = true;
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t kx = d.kids[n.a + 2 * order[j]];
        if (j + 1 < m && d.key_cmp(kx, d.kids[n.a + 2 * order[j + 1]]) == 0) continue;  // a later duplicate wins
        bool skipped = false;
        for (int s = 0; s < nskip && !skipped; s++) skipped = d.key_eq(kx, skip[s], strlen(skip[s]));
        if (skipped) continue;
        if (!first) out += '|';
        first = false;
        const JNode& k = d.nodes[kx];
        out.append(d.text, k.a, k.b - k.a);
        out += ':';
        ser(d, d.kids[n.a + 2 * order[j] + 1], out);
    }
}

void ser(const Doc& d, uint32_t x, std::string& out) {
    const JNode n = d.nodes[x];
    switch (n.k) {
        case J_NULL:
            return;
        case J_TRUE:
            out += "True";
            return;
        case J_FALSE:
            out += "False";
            return;
        case J_INT:
        case J_STR:
            out.append(d.text, n.a, n.b - n.a);
            return;
        case J_ARR:
            for (uint32_t i = n.a; i < n.b; i++) {
                if (i > n.a) out += ',';
                ser(d, d.kids[i], out);
            }
            return;
        case J_OBJ:
            ser_obj(d, n, out, nullptr, 0);
            return;
    }
}

const char* const kExcluded[3] = {"signature", "signatures", "fees"};  // client_authn.py:198

bool excluded(const char* s, size_t n) {
    for (const char* x : kExcluded)
        if (strlen(x) == n && memcmp(x, s, n) == 0) return true;
    return false;
}

// Request fields (request.py:16-39), looked up in the top-level dict (the last duplicate wins).
enum { F_IDR, F_REQID, F_OP, F_SIG, F_SIGS, F_PV, F_TAA, F_ENDORSER, F_NFIXED };
const char* const kFieldNames[F_NFIXED] = {"identifier", "reqId",           "operation",     "signature",
                                           "signatures", "protocolVersion", "taaAcceptance", "endorser"};

// PV_SER_REQUEST: M = serialize(as_dict minus excluded), digest = sha256(serialize(signingState())).
// Each field value is serialized once (into `piece`) and the two outputs are assembled from the
// pieces: the signed payload's members and the signing state's members, each in sorted name order.
struct Piece {
    const char* name;
    size_t len;
    uint32_t a, b;  // serialized value: piece[a, b)
};

void put_members(Piece* ps, int np, const std::string& piece, std::string& out) {
    for (int i = 1; i < np; i++) {  // insertion sort by name (a handful of members)
        Piece x = ps[i];
        int j = i;
        while (j > 0) {
            const int c = memcmp(x.name, ps[j - 1].name, std::min(x.len, ps[j - 1].len));
            if (c > 0 || (c == 0 && x.len >= ps[j - 1].len)) break;
            ps[j] = ps[j - 1];
            j--;
        }
        ps[j] = x;
    }
    for (int i = 0; i < np; i++) {
        if (i) out += '|';
        out.append(ps[i].name, ps[i].len);
        out += ':';
        out.append(piece, ps[i].a, ps[i].b - ps[i].a);
    }
}

int ser_request(Doc& d, uint32_t root, const std::vector<std::string>& plugins, std::string& out, uint8_t* digest,
                std::string& piece, std::string& state) {
    const JNode top = d.nodes[root];
    const size_t nf = F_NFIXED + plugins.size();
    auto name = [&](size_t f) { return f < F_NFIXED ? kFieldNames[f] : plugins[f - F_NFIXED].c_str(); };
    uint32_t val_small[F_NFIXED + 8];
    std::vector<uint32_t> val_big;
    uint32_t* val = val_small;
    if (nf > F_NFIXED + 8) {
        val_big.resize(nf);
        val = val_big.data();
    }
    for (size_t f = 0; f < nf; f++) val[f] = kBad;
    for (uint32_t i = top.a; i < top.b; i += 2) {
        const JNode& k = d.nodes[d.kids[i]];
        const size_t kl = k.b - k.a;
        for (size_t f = 0; f < nf; f++) {
            const char* nm = name(f);
            if (nm[0] == d.text[k.a] && strlen(nm) == kl && memcmp(d.text.data() + k.a, nm, kl) == 0) val[f] = d.kids[i + 1];
        }
    }
    auto present = [&](size_t f) { return val[f] != kBad && d.nodes[val[f]].k != J_NULL; };  // `is not None`
    piece.clear();
    auto make = [&](size_t f, uint32_t v) {  // serialize(value) once; kBad = None -> ""
        const uint32_t a = (uint32_t)piece.size();
        if (v != kBad) ser(d, v, piece);
        return Piece{name(f), strlen(name(f)), a, (uint32_t)piece.size()};
    };
    // as_dict (request.py:53-74), minus the keys excluded from signing
    std::vector<Piece> big_ps;
    Piece ps_small[F_NFIXED + 8];
    Piece* ps = ps_small;
    if (nf > F_NFIXED + 8) {
        big_ps.resize(nf + 2);
        ps = big_ps.data();
    }
    int np = 0;
    Piece pv[F_NFIXED];
    bool have[F_NFIXED] = {false};
    pv[F_REQID] = make(F_REQID, val[F_REQID]);
    pv[F_OP] = make(F_OP, val[F_OP]);
    have[F_REQID] = have[F_OP] = true;
    ps[np++] = pv[F_REQID];
    ps[np++] = pv[F_OP];
    for (int f : {F_IDR, F_PV, F_TAA, F_ENDORSER})  // signature(s) are excluded from the payload
        if (present(f)) {
            pv[f] = make(f, val[f]);
            have[f] = true;
            ps[np++] = pv[f];
        }
    std::vector<Piece> plug;
    for (size_t f = F_NFIXED; f < nf; f++)  // plugin fields: hasattr -> given as a keyword
        if (val[f] != kBad) {
            Piece x = make(f, val[f]);
            plug.push_back(x);
            if (!excluded(x.name, x.len)) ps[np++] = x;
        }
    put_members(ps, np, piece, out);
    if (!digest) return PV_SER_OK;
    // signingState (request.py:95-121); identifier = _identifier or ",".join(sorted(signatures))
    np = 0;
    if (val[F_IDR] != kBad && d.truthy(val[F_IDR])) {
        ps[np++] = have[F_IDR] ? pv[F_IDR] : make(F_IDR, val[F_IDR]);
    } else if (val[F_SIGS] != kBad && d.truthy(val[F_SIGS])) {
        const JNode s = d.nodes[val[F_SIGS]];
        if (s.k != J_OBJ) return PV_SER_DEFER;  // .keys() of a non-dict raises in Python
        std::vector<uint32_t> keys;
        for (uint32_t i = s.a; i < s.b; i += 2) keys.push_back(d.kids[i]);
        std::sort(keys.begin(), keys.end(), [&](uint32_t x, uint32_t y) { return d.key_cmp(x, y) < 0; });
        keys.erase(std::unique(keys.begin(), keys.end(), [&](uint32_t x, uint32_t y) { return d.key_cmp(x, y) == 0; }),
                   keys.end());
        const uint32_t a = (uint32_t)piece.size();
        for (size_t i = 0; i < keys.size(); i++) {
            if (i) piece += ',';
            const JNode k = d.nodes[keys[i]];
            piece.append(d.text, k.a, k.b - k.a);
        }
        ps[np++] = Piece{name(F_IDR), strlen(name(F_IDR)), a, (uint32_t)piece.size()};
    } else {
        ps[np++] = make(F_IDR, kBad);
    }
    ps[np++] = pv[F_REQID];
    ps[np++] = pv[F_OP];
    for (int f : {F_PV, F_TAA, F_ENDORSER, F_SIGS, F_SIG})
        if (present(f)) ps[np++] = have[f] ? pv[f] : make(f, val[f]);
    for (const Piece& x : plug)  // plugin fields: included when truthy
        for (size_t f = F_NFIXED; f < nf; f++)
            if (name(f) == x.name && d.truthy(val[f])) ps[np++] = x;
    state.clear();
    put_members(ps, np, piece, state);
    sha256(reinterpret_cast<const uint8_t*>(state.data()), state.size(), digest);
    return PV_SER_OK;
}

int serialize_one(const uint8_t* js, size_t n, int mode, const std::vector<std::string>& plugins, Doc& d,
                  std::string& out, uint8_t* digest, std::string& piece, std::string& state) {
    uint32_t root = 0;
    const int st = parse(js, n, d, root);
    if (st != PV_SER_OK) return st;
    if (d.nodes[root].k != J_OBJ) return PV_SER_NOT_OBJECT;
    if (mode == PV_SER_DICT) {
        ser_obj(d, d.nodes[root], out, nullptr, 0);
        return PV_SER_OK;
    }
    if (mode == PV_SER_AUTHN) {
        ser_obj(d, d.nodes[root], out, kExcluded, 3);
        return PV_SER_OK;
    }
    return ser_request(d, root, plugins, out, digest, piece, state);
}

// ------------------------------------------------------------------------------ wire planning
// The signature plan of one parsed request (pv_wire_plan): what CoreAuthMixin._select_signatures
// (client_authn.py:240-264) returns for Request(**msg).as_dict, restricted to the cases whose
// Python result this code reproduces exactly; everything else is PV_PLAN_PY.

// A non-empty string of printable, non-space ASCII: what wire.py's _plain accepts (ASCII, nothing
// str.rstrip() would strip), narrowed so that the text needs no decoding or stripping anywhere
// (base58 identifiers and signatures always qualify; anything else takes the Python path).
bool plain_text(const Doc& d, uint32_t node) {
    const JNode& x = d.nodes[node];
    if (x.k != J_STR || x.b == x.a) return false;
    for (uint32_t i = x.a; i < x.b; i++) {
        const uint8_t c = (uint8_t)d.text[i];
        if (c <= 0x20 || c >= 0x7F) return false;
    }
    return true;
}

struct PlanOut {  // one thread's share of the plan
    std::vector<uint8_t> kind;
    std::vector<uint32_t> type_local, npairs, pair_local;
    std::vector<uint64_t> sig_len;
    std::string sigs;
    std::deque<std::string> names, types;  // local first-appearance order (stable addresses)
    std::unordered_map<std::string_view, uint32_t> name_id, type_id;
    uint32_t last_type = kBad;
};

uint32_t local_id(std::unordered_map<std::string_view, uint32_t>& m, std::deque<std::string>& v, const std::string& t,
                  uint32_t a, uint32_t b) {
    const std::string_view s(t.data() + a, b - a);
    auto it = m.find(s);
    if (it != m.end()) return it->second;
    const uint32_t id = (uint32_t)v.size();
    v.emplace_back(s);
    m.emplace(std::string_view(v.back()), id);
    return id;
}

// last value of top-level key `name` (a Python dict keeps the last duplicate), or kBad
uint32_t member(const Doc& d, const JNode obj, const char* name) {
    uint32_t v = kBad;
    const size_t len = strlen(name);
    for (uint32_t i = obj.a; i < obj.b; i += 2)
        if (d.key_eq(d.kids[i], name, len)) v = d.kids[i + 1];
    return v;
}

void plan_one(const Doc& d, uint32_t root, bool plugins, PlanOut& o) {
    const size_t p0 = o.pair_local.size(), s0 = o.sigs.size(), l0 = o.sig_len.size();
    auto py = [&]() {
        o.pair_local.resize(p0);
        o.sigs.resize(s0);
        o.sig_len.resize(l0);
        o.kind.push_back(PV_PLAN_PY);
        o.type_local.push_back(0);
        o.npairs.push_back(0);
    };
    const JNode top = d.nodes[root];
    if (plugins || member(d, top, "self") != kBad) return py();  // Request(**msg) itself decides
    const uint32_t op = member(d, top, "operation");
    if (op == kBad || d.nodes[op].k != J_OBJ) return py();
    const uint32_t typ = member(d, d.nodes[op], "type");
    if (typ == kBad || d.nodes[typ].k != J_STR) return py();
    const uint32_t idr = member(d, top, "identifier"), sig = member(d, top, "signature"),
                   sigs = member(d, top, "signatures");
    auto is_null = [&](uint32_t v) { return v == kBad || d.nodes[v].k == J_NULL; };
    if (is_null(sig) && is_null(sigs)) return py();  // MissingSignature
    auto add_pair = [&](uint32_t name, uint32_t s) {
        const JNode& n = d.nodes[name];
        o.pair_local.push_back(local_id(o.name_id, o.names, d.text, n.a, n.b));
        const JNode& x = d.nodes[s];
        o.sigs.append(d.text, x.a, x.b - x.a);
        o.sig_len.push_back(x.b - x.a);
    };
    uint8_t kind;
    if (idr != kBad && d.truthy(idr) && sig != kBad && d.truthy(sig)) {
        if (!plain_text(d, idr) || !plain_text(d, sig)) return py();
        add_pair(idr, sig);
        kind = PV_PLAN_SINGLE;
    } else {
        if (!is_null(sig) || sigs == kBad) return py();  // the cache would store a non-None signature
        const JNode s = d.nodes[sigs];
        if (s.k != J_OBJ || s.b == s.a) return py();
        for (uint32_t i = s.a; i < s.b; i += 2) {
            const uint32_t k = d.kids[i], v = d.kids[i + 1];
            if (!plain_text(d, k) || !plain_text(d, v)) return py();
            for (uint32_t j = s.a; j < i; j += 2)  // duplicate names: dict order rules, left to Python
                if (d.key_cmp(d.kids[j], k) == 0) return py();
            add_pair(k, v);
        }
        kind = PV_PLAN_MULTI;
    }
    const JNode& t = d.nodes[typ];
    o.kind.push_back(kind);
    const uint32_t lt = o.last_type;  // consecutive requests mostly share their txn type
    if (lt != kBad && o.types[lt].size() == t.b - t.a && memcmp(o.types[lt].data(), d.text.data() + t.a, t.b - t.a) == 0)
        o.type_local.push_back(lt);
    else
        o.type_local.push_back(o.last_type = local_id(o.type_id, o.types, d.text, t.a, t.b));
    o.npairs.push_back((uint32_t)(o.pair_local.size() - p0));
}

}  // namespace

extern "C" int pv_wire_plan(const char* json, const uint64_t* off, uint64_t n, const char* plugin_fields, int threads,
                            PvWirePlan* P) {
    if (!P) return pv_fail(PV_ERR_ARG, "pv_wire_plan: null plan");
    P->n_pairs = P->n_names = P->n_types = 0;
    if (n == 0) {
        if (P->msg_off) P->msg_off[0] = 0;
        if (P->pair_off) P->pair_off[0] = 0;
        if (P->sig_off) P->sig_off[0] = 0;
        if (P->name_off) P->name_off[0] = 0;
        if (P->type_off) P->type_off[0] = 0;
        return PV_OK;
    }
    if (!json || !off || !P->msg_off || !P->status || !P->digest || !P->kind || !P->type_id || !P->pair_off ||
        !P->pair_name || !P->sig_off || !P->name_off || !P->type_off || (P->msg_cap && !P->msg_out) ||
        (P->sigs_cap && !P->sigs) || (P->names_cap && !P->names) || (P->types_cap && !P->types))
        return pv_fail(PV_ERR_ARG, "pv_wire_plan: null pointer");
    for (uint64_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) return pv_fail(PV_ERR_ARG, "pv_wire_plan: offsets must be non-decreasing");
    std::vector<std::string> plugins;
    if (plugin_fields)
        for (const char* q = plugin_fields; *q; q += strlen(q) + 1) plugins.emplace_back(q);
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(threads, 1), (n + 255) / 256));
    std::vector<std::string> outs(T);
    std::vector<std::vector<uint64_t>> lens(T);
    std::vector<PlanOut> plans(T);
    auto work = [&](int t) {
        const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
        Doc d;
        std::string piece, state;
        std::string& out = outs[t];
        PlanOut& po = plans[t];
        lens[t].resize(hi - lo);
        out.reserve(off[hi] - off[lo] + 64);  // a signing message is never longer than its JSON text
        po.sigs.reserve((off[hi] - off[lo]) / 4);
        po.kind.reserve(hi - lo);
        po.type_local.reserve(hi - lo);
        po.npairs.reserve(hi - lo);
        po.pair_local.reserve(hi - lo);
        po.sig_len.reserve(hi - lo);
        for (uint64_t i = lo; i < hi; i++) {
            const size_t before = out.size();
            uint8_t* dg = P->digest + 32 * i;
            uint32_t root = 0;
            int st = parse(reinterpret_cast<const uint8_t*>(json) + off[i], (size_t)(off[i + 1] - off[i]), d, root);
            if (st == PV_SER_OK && d.nodes[root].k != J_OBJ) st = PV_SER_NOT_OBJECT;
            if (st == PV_SER_OK) st = ser_request(d, root, plugins, out, dg, piece, state);
            if (st != PV_SER_OK) {
                out.resize(before);
                memset(dg, 0, 32);
                po.kind.push_back(PV_PLAN_PY);
                po.type_local.push_back(0);
                po.npairs.push_back(0);
            } else {
                plan_one(d, root, !plugins.empty(), po);
            }
            P->status[i] = (uint8_t)st;
            lens[t][i - lo] = out.size() - before;
        }
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++) th.emplace_back(work, t);
        for (auto& x : th) x.join();
    }
    // sizes first: nothing is written past a capacity
    uint64_t total = 0, npairs = 0, nsig = 0;
    for (int t = 0; t < T; t++) {
        total += outs[t].size();
        npairs += plans[t].pair_local.size();
        nsig += plans[t].sigs.size();
    }
    if (total > P->msg_cap) {
        P->msg_off[n] = total;
        return pv_fail(PV_ERR_ARG, "pv_wire_plan: msg_cap too small (msg_off[n] = bytes needed)");
    }
    if (npairs > P->pair_cap || nsig > P->sigs_cap) return pv_fail(PV_ERR_ARG, "pv_wire_plan: pair/sig capacity too small");
    // distinct identifiers and types over the whole batch, in first-appearance order
    std::unordered_map<std::string, uint32_t> gname, gtype;
    std::vector<const std::string*> names, types;
    std::vector<std::vector<uint32_t>> name_map(T), type_map(T);
    for (int t = 0; t < T; t++) {
        for (const std::string& s : plans[t].names) {
            auto it = gname.emplace(s, (uint32_t)names.size());
            if (it.second) names.push_back(&it.first->first);
            name_map[t].push_back(it.first->second);
        }
        for (const std::string& s : plans[t].types) {
            auto it = gtype.emplace(s, (uint32_t)types.size());
            if (it.second) types.push_back(&it.first->first);
            type_map[t].push_back(it.first->second);
        }
    }
    uint64_t nb = 0, tb = 0;
    for (auto* s : names) nb += s->size();
    for (auto* s : types) tb += s->size();
    if (nb > P->names_cap || names.size() > P->pair_cap || tb > P->types_cap || types.size() > n)
        return pv_fail(PV_ERR_ARG, "pv_wire_plan: name/type capacity too small");
    uint64_t pos = 0, i = 0, pp = 0, sp = 0;
    for (int t = 0; t < T; t++) {
        const PlanOut& po = plans[t];
        if (!outs[t].empty()) memcpy(P->msg_out + pos, outs[t].data(), outs[t].size());
        if (!po.sigs.empty()) memcpy(P->sigs + sp, po.sigs.data(), po.sigs.size());
        uint64_t q = 0;
        for (size_t k = 0; k < lens[t].size(); k++, i++) {
            P->msg_off[i] = pos;
            pos += lens[t][k];
            P->kind[i] = po.kind[k];
            P->type_id[i] = po.kind[k] == PV_PLAN_PY ? 0 : type_map[t][po.type_local[k]];
            P->pair_off[i] = pp;
            for (uint32_t j = 0; j < po.npairs[k]; j++, q++, pp++) {
                P->pair_name[pp] = name_map[t][po.pair_local[q]];
                P->sig_off[pp] = sp;
                sp += po.sig_len[q];
            }
        }
    }
    P->msg_off[n] = pos;
    P->pair_off[n] = pp;
    P->sig_off[pp] = sp;
    if (P->sig_lines) {  // the same texts newline-terminated (one split gives every signature)
        for (uint64_t q = 0; q < pp; q++) {
            const uint64_t a = P->sig_off[q], b = P->sig_off[q + 1];
            memcpy(P->sig_lines + a + q, P->sigs + a, b - a);
            P->sig_lines[b + q] = '\n';
        }
    }
    if (P->keys_hex) {
        static const char hx[] = "0123456789abcdef";
        auto hex_rows = [&](uint64_t lo, uint64_t hi) {
            for (uint64_t r = lo; r < hi; r++) {
                char* o = P->keys_hex + 65 * r;
                const uint8_t* g = P->digest + 32 * r;
                for (int k = 0; k < 32; k++) {
                    o[2 * k] = hx[g[k] >> 4];
                    o[2 * k + 1] = hx[g[k] & 15];
                }
                o[64] = '\n';
            }
        };
        if (T == 1) {
            hex_rows(0, n);
        } else {
            std::vector<std::thread> th;
            for (int t = 0; t < T; t++) th.emplace_back(hex_rows, n * t / T, n * (t + 1) / T);
            for (auto& x : th) x.join();
        }
    }
    uint64_t o = 0;
    for (size_t k = 0; k < names.size(); k++) {
        P->name_off[k] = o;
        if (!names[k]->empty()) memcpy(P->names + o, names[k]->data(), names[k]->size());
        o += names[k]->size();
    }
    P->name_off[names.size()] = o;
    o = 0;
    for (size_t k = 0; k < types.size(); k++) {
        P->type_off[k] = o;
        if (!types[k]->empty()) memcpy(P->types + o, types[k]->data(), types[k]->size());
        o += types[k]->size();
    }
    P->type_off[types.size()] = o;
    P->n_pairs = pp;
    P->n_names = names.size();
    P->n_types = types.size();
    return PV_OK;
}

extern "C" int pv_signing_serialize_json(const char* json, const uint64_t* off, uint64_t n, int mode,
                                         const char* plugin_fields, int threads, uint8_t* msg_out, uint64_t msg_cap,
                                         uint64_t* msg_off, uint8_t* digest, uint8_t* status) {
    if (n == 0) {
        if (msg_off) msg_off[0] = 0;
        return PV_OK;
    }
    if (!json || !off || !msg_off || !status || (msg_cap && !msg_out))
        return pv_fail(PV_ERR_ARG, "pv_signing_serialize_json: null pointer");
    if (mode != PV_SER_DICT && mode != PV_SER_AUTHN && mode != PV_SER_REQUEST)
        return pv_fail(PV_ERR_ARG, "pv_signing_serialize_json: unknown mode");
    for (uint64_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) return pv_fail(PV_ERR_ARG, "pv_signing_serialize_json: offsets must be non-decreasing");
    std::vector<std::string> plugins;
    if (plugin_fields)
        for (const char* q = plugin_fields; *q; q += strlen(q) + 1) plugins.emplace_back(q);
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(threads, 1), (n + 255) / 256));
    std::vector<std::string> outs(T);
    std::vector<std::vector<uint64_t>> lens(T);
    auto work = [&](int t) {
        const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
        Doc d;
        std::string piece, state;
        std::string& out = outs[t];
        lens[t].resize(hi - lo);
        for (uint64_t i = lo; i < hi; i++) {
            const size_t before = out.size();
            uint8_t* dg = (mode == PV_SER_REQUEST && digest) ? digest + 32 * i : nullptr;
            const int st = serialize_one(reinterpret_cast<const uint8_t*>(json) + off[i], (size_t)(off[i + 1] - off[i]),
                                         mode, plugins, d, out, dg, piece, state);
            if (st != PV_SER_OK) {
                out.resize(before);
                if (dg) memset(dg, 0, 32);
            }
            status[i] = (uint8_t)st;
            lens[t][i - lo] = out.size() - before;
        }
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++) th.emplace_back(work, t);
        for (auto& x : th) x.join();
    }
    uint64_t total = 0;
    for (int t = 0; t < T; t++) total += outs[t].size();
    if (total > msg_cap) {
        msg_off[n] = total;
        return pv_fail(PV_ERR_ARG, "pv_signing_serialize_json: msg_cap too small (msg_off[n] = bytes needed)");
    }
    uint64_t pos = 0, i = 0;
    for (int t = 0; t < T; t++) {
        if (!outs[t].empty()) memcpy(msg_out + pos, outs[t].data(), outs[t].size());
        for (uint64_t len : lens[t]) {
            msg_off[i++] = pos;
            pos += len;
        }
    }
    msg_off[n] = pos;
    return PV_OK;
}
