// Host-side batch preparation for the verify engine (C++, no GPU):
//   pv_b58decode_batch   base58.b58decode semantics (PyPI base58 2.x; reference calls at
//                        plenum/server/client_authn.py:97 and plenum/common/verifier.py:27,37,50)
//   pv_b58encode         base58.b58encode (verifier.py:37 re-encodes the expanded verkey)
//   pv_resolve_verkeys   DidVerifier.__init__ + verkey setter (plenum/common/verifier.py:24-50) and
//                        stp_core Verifier/VerifyKey key decoding (stp_core/crypto/nacl_wrappers.py:
//                        62-84, 212-229), batched.
// Inputs are byte strings. The Python layer applies str-level rules (str.rstrip() of Unicode
// whitespace, ASCII encoding errors) before calling in; here trailing ASCII whitespace is stripped,
// which is what bytes.rstrip() does.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/plenum_verify.h"

namespace {

const char* kAlphabet = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

struct B58Map {
    int8_t v[256];
    B58Map() {
        memset(v, -1, sizeof v);
        for (int i = 0; i < 58; i++) v[(unsigned char)kAlphabet[i]] = (int8_t)i;
    }
};
const B58Map kMap;

inline bool is_ascii_ws(unsigned char c) { return c == ' ' || (c >= 9 && c <= 13); }

// Decode s[0..len) into out (big-endian bytes). Returns 0 ok, 1 invalid character, 2 too long.
int b58decode_one(const unsigned char* s, size_t len, std::vector<uint8_t>& out) {
    while (len > 0 && is_ascii_ws(s[len - 1])) len--;
    size_t zeros = 0;
    while (zeros < len && s[zeros] == '1') zeros++;
    // little-endian accumulator of the integer value of s[zeros..len)
    std::vector<uint8_t> acc;
    acc.reserve(len);
    for (size_t i = zeros; i < len; i++) {
        const int d = kMap.v[s[i]];
        if (d < 0) return 1;
        uint32_t carry = (uint32_t)d;
        for (size_t j = 0; j < acc.size(); j++) {
            carry += 58u * acc[j];
            acc[j] = (uint8_t)carry;
            carry >>= 8;
        }
        while (carry) {
            acc.push_back((uint8_t)carry);
            carry >>= 8;
        }
    }
    out.assign(zeros, 0);
    for (size_t j = acc.size(); j > 0; j--) out.push_back(acc[j - 1]);
    return 0;
}

int hexval(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

// stp_core Verifier(key) on raw bytes: 32 bytes -> raw key; otherwise VerifyKey(key, HexEncoder):
// binascii.unhexlify(key) must give exactly 32 bytes. Returns 0 ok, 2 InvalidKey, 3 no key.
int nacl_key_from_bytes(const std::vector<uint8_t>& raw, uint8_t pk[32]) {
    if (raw.empty()) return 3;
    if (raw.size() == 32) {
        memcpy(pk, raw.data(), 32);
        return 0;
    }
    if (raw.size() != 64) return 2;  // odd length or wrong decoded size -> ValueError
    for (int i = 0; i < 32; i++) {
        const int hi = hexval(raw[2 * i]), lo = hexval(raw[2 * i + 1]);
        if (hi < 0 || lo < 0) return 2;
        pk[i] = (uint8_t)(hi * 16 + lo);
    }
    return 0;
}

}  // namespace

extern "C" {

int pv_b58decode_batch(const char* chars, const uint64_t* off, uint64_t n, uint8_t* out, uint64_t out_stride,
                       uint32_t* out_len, uint8_t* status) {
    if (n == 0) return PV_OK;
    if (!chars || !off || !out || !out_len || !status) return PV_ERR_ARG;
    std::vector<uint8_t> buf;
    for (uint64_t i = 0; i < n; i++) {
        const unsigned char* s = reinterpret_cast<const unsigned char*>(chars) + off[i];
        const int rc = b58decode_one(s, (size_t)(off[i + 1] - off[i]), buf);
        out_len[i] = 0;
        if (rc) {
            status[i] = (uint8_t)rc;
            continue;
        }
        if (buf.size() > out_stride) {
            status[i] = 2;
            out_len[i] = (uint32_t)buf.size();
            continue;
        }
        memcpy(out + i * out_stride, buf.data(), buf.size());
        out_len[i] = (uint32_t)buf.size();
        status[i] = 0;
    }
    return PV_OK;
}

// base58.b58encode: leading 0x00 bytes -> '1', then the base-58 digits of the integer value.
// Writes at most cap chars; returns the encoded length (which may exceed cap) or a negative error.
int64_t pv_b58encode(const uint8_t* data, uint64_t len, char* out, uint64_t cap) {
    uint64_t zeros = 0;
    while (zeros < len && data[zeros] == 0) zeros++;
    std::vector<uint8_t> digits;  // little-endian base-58 digits
    for (uint64_t i = zeros; i < len; i++) {
        uint32_t carry = data[i];
        for (size_t j = 0; j < digits.size(); j++) {
            carry += (uint32_t)digits[j] << 8;
            digits[j] = (uint8_t)(carry % 58);
            carry /= 58;
        }
        while (carry) {
            digits.push_back((uint8_t)(carry % 58));
            carry /= 58;
        }
    }
    const uint64_t total = zeros + digits.size();
    if (out) {
        uint64_t p = 0;
        for (uint64_t i = 0; i < zeros && p < cap; i++) out[p++] = '1';
        for (size_t j = digits.size(); j > 0 && p < cap; j--) out[p++] = kAlphabet[digits[j - 1]];
    }
    return (int64_t)total;
}

int pv_resolve_verkeys(const char* idr_chars, const uint64_t* idr_off, const char* vk_chars, const uint64_t* vk_off,
                       const uint8_t* has_verkey, uint64_t n, uint8_t* pk_out, uint8_t* status) {
    if (n == 0) return PV_OK;
    if (!idr_chars || !idr_off || !vk_chars || !vk_off || !has_verkey || !pk_out || !status) return PV_ERR_ARG;
    std::vector<uint8_t> idr_raw, vk_raw, tail;
    for (uint64_t i = 0; i < n; i++) {
        const unsigned char* idr = reinterpret_cast<const unsigned char*>(idr_chars) + idr_off[i];
        const size_t idr_len = (size_t)(idr_off[i + 1] - idr_off[i]);
        const unsigned char* vk = reinterpret_cast<const unsigned char*>(vk_chars) + vk_off[i];
        const size_t vk_len = (size_t)(vk_off[i + 1] - vk_off[i]);
        uint8_t* pk = pk_out + 32 * i;
        memset(pk, 0, 32);
        bool vk_present = has_verkey[i] != 0;
        bool vk_truthy = vk_present && vk_len > 0;
        // the resolved raw key bytes (what the setter's b58decode(value) will produce)
        bool use_idr_as_vk = false;
        if (idr_len > 0) {  // `if identifier:`
            if (b58decode_one(idr, idr_len, idr_raw) != 0) {
                status[i] = 4;  // ValueError from b58decode(identifier) propagates
                continue;
            }
            if (idr_raw.size() == 32 && !vk_truthy) use_idr_as_vk = true;  // cryptonym
            if (!vk_truthy && !use_idr_as_vk) {
                status[i] = 1;
                continue;
            }
            if (!use_idr_as_vk && vk[0] == '~') {
                if (b58decode_one(vk + 1, vk_len - 1, tail) != 0) {
                    status[i] = 4;  // ValueError from b58decode(verkey[1:]) propagates
                    continue;
                }
                // b58encode(idr_raw + tail) then the setter's b58decode: a byte-exact round trip
                vk_raw = idr_raw;
                vk_raw.insert(vk_raw.end(), tail.begin(), tail.end());
                status[i] = (uint8_t)nacl_key_from_bytes(vk_raw, pk);
                continue;
            }
        }
        // setter: NaclVerifier(b58decode(value))
        if (use_idr_as_vk) {
            status[i] = (uint8_t)nacl_key_from_bytes(idr_raw, pk);
            continue;
        }
        if (!vk_present) {  // b58decode(None) -> AttributeError -> InvalidKey
            status[i] = 2;
            continue;
        }
        if (b58decode_one(vk, vk_len, vk_raw) != 0) {
            status[i] = 2;
            continue;
        }
        status[i] = (uint8_t)nacl_key_from_bytes(vk_raw, pk);
    }
    return PV_OK;
}

}  // extern "C"
