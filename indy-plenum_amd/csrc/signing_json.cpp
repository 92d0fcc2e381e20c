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
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
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

void sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t i = 0;
    for (; i + 64 <= len; i += 64) sha256_compress(st, data + i);
    uint8_t tail[128] = {0};
    const size_t rem = len - i;
    memcpy(tail, data + i, rem);
    tail[rem] = 0x80;
    const size_t tl = rem + 9 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)len * 8;
    for (int k = 0; k < 8; k++) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
    sha256_compress(st, tail);
    if (tl == 128) sha256_compress(st, tail + 64);
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
struct Member {  // one (name, value) of a dict synthesized from the request's fields
    const char* name;
    size_t len;
    uint32_t value;
};

void ser(const Doc& d, uint32_t x, std::string& out);

// dict: keys deduplicated (the last value wins, as in a Python dict), sorted by code point (= UTF-8
// byte order), "k:v" joined by "|"; `skip` lists top-level keys to leave out.
void ser_obj(const Doc& d, const JNode n, std::string& out, const char* const* skip, int nskip) {
    const uint32_t m = (n.b - n.a) / 2;
    std::vector<uint32_t> order(m);
    for (uint32_t i = 0; i < m; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
        return d.key_cmp(d.kids[n.a + 2 * x], d.kids[n.a + 2 * y]) < 0;
    });
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

void ser_members(const Doc& d, std::vector<Member>& ms, std::string& out) {
    std::sort(ms.begin(), ms.end(), [](const Member& x, const Member& y) {
        const int c = memcmp(x.name, y.name, std::min(x.len, y.len));
        return c ? c < 0 : x.len < y.len;
    });
    for (size_t i = 0; i < ms.size(); i++) {
        if (i) out += '|';
        out.append(ms[i].name, ms[i].len);
        out += ':';
        ser(d, ms[i].value, out);
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
int ser_request(Doc& d, uint32_t root, const std::vector<std::string>& plugins, std::string& out, uint8_t* digest) {
    const JNode top = d.nodes[root];
    const size_t nf = F_NFIXED + plugins.size();
    auto name = [&](size_t f) { return f < F_NFIXED ? kFieldNames[f] : plugins[f - F_NFIXED].c_str(); };
    std::vector<uint32_t> val(nf, kBad);
    for (uint32_t i = top.a; i < top.b; i += 2)
        for (size_t f = 0; f < nf; f++)
            if (d.key_eq(d.kids[i], name(f), strlen(name(f)))) val[f] = d.kids[i + 1];
    const uint32_t none = d.add(J_NULL);
    auto present = [&](size_t f) { return val[f] != kBad && d.nodes[val[f]].k != J_NULL; };  // `is not None`
    auto field = [&](size_t f) { return val[f] == kBad ? none : val[f]; };
    auto member = [&](size_t f, uint32_t v) { return Member{name(f), strlen(name(f)), v}; };
    // as_dict (request.py:53-74), minus the keys excluded from signing
    std::vector<Member> ms;
    ms.push_back(member(F_REQID, field(F_REQID)));
    ms.push_back(member(F_OP, field(F_OP)));
    for (int f : {F_IDR, F_SIGS, F_SIG, F_PV, F_TAA, F_ENDORSER})
        if (present(f)) ms.push_back(member(f, val[f]));
    for (size_t f = F_NFIXED; f < nf; f++)  // plugin fields: hasattr -> given as a keyword
        if (val[f] != kBad) ms.push_back(member(f, val[f]));
    std::vector<Member> signed_ms;
    for (const Member& m : ms)
        if (!excluded(m.name, m.len)) signed_ms.push_back(m);
    ser_members(d, signed_ms, out);
    if (!digest) return PV_SER_OK;
    // signingState (request.py:95-121); identifier = _identifier or ",".join(sorted(signatures))
    uint32_t idr = none;
    if (val[F_IDR] != kBad && d.truthy(val[F_IDR])) {
        idr = val[F_IDR];
    } else if (val[F_SIGS] != kBad && d.truthy(val[F_SIGS])) {
        const JNode s = d.nodes[val[F_SIGS]];
        if (s.k != J_OBJ) return PV_SER_DEFER;  // .keys() of a non-dict raises in Python
        std::vector<uint32_t> keys;
        for (uint32_t i = s.a; i < s.b; i += 2) keys.push_back(d.kids[i]);
        std::sort(keys.begin(), keys.end(), [&](uint32_t x, uint32_t y) { return d.key_cmp(x, y) < 0; });
        keys.erase(std::unique(keys.begin(), keys.end(), [&](uint32_t x, uint32_t y) { return d.key_cmp(x, y) == 0; }),
                   keys.end());
        std::string joined;
        for (size_t i = 0; i < keys.size(); i++) {
            if (i) joined += ',';
            const JNode k = d.nodes[keys[i]];
            joined.append(d.text, k.a, k.b - k.a);
        }
        idr = d.add_text(J_STR, joined.data(), joined.size());
    }
    std::vector<Member> st;
    st.push_back(member(F_IDR, idr));
    st.push_back(member(F_REQID, field(F_REQID)));
    st.push_back(member(F_OP, field(F_OP)));
    for (int f : {F_PV, F_TAA, F_ENDORSER, F_SIGS, F_SIG})
        if (present(f)) st.push_back(member(f, val[f]));
    for (size_t f = F_NFIXED; f < nf; f++)  // plugin fields: included when truthy
        if (val[f] != kBad && d.truthy(val[f])) st.push_back(member(f, val[f]));
    std::string s;
    ser_members(d, st, s);
    sha256(reinterpret_cast<const uint8_t*>(s.data()), s.size(), digest);
    return PV_SER_OK;
}

int serialize_one(const uint8_t* js, size_t n, int mode, const std::vector<std::string>& plugins, Doc& d,
                  std::string& out, uint8_t* digest) {
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
    return ser_request(d, root, plugins, out, digest);
}

}  // namespace

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
        std::string& out = outs[t];
        lens[t].resize(hi - lo);
        for (uint64_t i = lo; i < hi; i++) {
            const size_t before = out.size();
            uint8_t* dg = (mode == PV_SER_REQUEST && digest) ? digest + 32 * i : nullptr;
            const int st = serialize_one(reinterpret_cast<const uint8_t*>(json) + off[i], (size_t)(off[i + 1] - off[i]),
                                         mode, plugins, d, out, dg);
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
