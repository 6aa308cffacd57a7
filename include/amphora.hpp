// C++17 host-side mirror of the reference's Java interface over the C ABI
// (include/amphora.h).  Header-only; link against libamphora_hip.so.
//
//   amphora::client::SecretShareUtil       <- amphora-java-client/.../client/SecretShareUtil.java:33-157
//   amphora::client::verifyOutputDeliveryObjects / maskSecret
//                                          <- DefaultAmphoraClient.java:150-160,476-505
//   amphora::service::SecretShareUtil      <- amphora-service/.../calculation/SecretShareUtil.java:30-107
//   amphora::service::OutputDeliveryService<- amphora-service/.../calculation/OutputDeliveryService.java:57-286
//   amphora::OutputDeliveryObject          <- amphora-common/.../OutputDeliveryObject.java:55-106
//   amphora::wire (base64, FactorPair JSON) <- Jackson on VerifiableSecretShare /
//                                             MultiplicationExchangeObject.java:20-39
//   amphora::nameUUIDFromBytes             <- java.util.UUID.nameUUIDFromBytes (MD5, version 3)
//
// Java BigIntegers become `amphora::u128` canonical integers (callers reduce
// arbitrary-size values mod p before constructing them; `fromDecimal` does
// that for decimal strings like the MAC key property).  Exceptions carry the
// reference's messages.  Every word of arithmetic runs on the GPU.
#ifndef AMPHORA_HPP_
#define AMPHORA_HPP_

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <exception>
#include <functional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "amphora.h"

namespace amphora {

using u128 = unsigned __int128;
using Bytes = std::vector<uint8_t>;

struct IntegrityVerificationException : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct IllegalArgumentException : std::invalid_argument {
  using std::invalid_argument::invalid_argument;
};
struct AmphoraServiceException : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct AmphoraClientException : std::runtime_error {  // amphora-common AmphoraClientException
  using std::runtime_error::runtime_error;
};
struct NativeError : std::runtime_error {
  int status;
  NativeError(int st, const std::string& m) : std::runtime_error(m), status(st) {}
};
// java.lang.ArrayIndexOutOfBoundsException: a ragged party's word starts past
// its array's end (recombineObject's Arrays.copyOfRange, AMPH_E_RANGE)
struct ArrayIndexOutOfBoundsException : std::out_of_range {
  using std::out_of_range::out_of_range;
};

inline void check(int st) {
  if (st == AMPH_E_RANGE) throw ArrayIndexOutOfBoundsException(amph_last_error());
  if (st != AMPH_OK) throw NativeError(st, std::string(amph_strerror(st)) + ": " + amph_last_error());
}

// java.util.Arrays.copyOfRange(byte[], from, to): zero-padded past the end,
// ArrayIndexOutOfBoundsException when `from` is past it
inline std::vector<uint8_t> copyOfRange(const std::vector<uint8_t>& a, size_t from, size_t to) {
  if (from > a.size()) throw ArrayIndexOutOfBoundsException("copyOfRange: from past the end of the array");
  std::vector<uint8_t> out(to - from, 0);
  std::copy(a.begin() + from, a.begin() + std::min(a.size(), to), out.begin());
  return out;
}

inline void storeLe(u128 x, uint8_t* out) {
  for (int i = 0; i < 16; ++i) out[i] = (uint8_t)(x >> (8 * i));
}
inline u128 loadLe(const uint8_t* in) {
  u128 x = 0;
  for (int i = 15; i >= 0; --i) x = (x << 8) | in[i];
  return x;
}
inline std::string toDecimal(u128 x) {
  if (x == 0) return "0";
  std::string s;
  while (x) {
    s.insert(s.begin(), char('0' + int(x % 10)));
    x /= 10;
  }
  return s;
}
// (a + b) mod p for a, b < p (129-bit intermediate)
inline u128 addMod(u128 a, u128 b, u128 p) {
  u128 s = a + b;
  if (s < a || s >= p) s -= p;
  return s;
}
// new BigInteger(decimal).mod(p): optional leading '-'
inline u128 fromDecimal(const std::string& dec, u128 p) {
  size_t i = 0;
  bool neg = !dec.empty() && dec[0] == '-';
  if (neg || (!dec.empty() && dec[0] == '+')) i = 1;
  if (i >= dec.size()) throw std::invalid_argument("Zero length BigInteger");
  u128 x = 0;
  for (; i < dec.size(); ++i) {
    if (dec[i] < '0' || dec[i] > '9') throw std::invalid_argument("For input string: \"" + dec + "\"");
    u128 x2 = addMod(x, x, p), x4 = addMod(x2, x2, p), x8 = addMod(x4, x4, p);
    x = addMod(addMod(x8, x2, p), (u128)(dec[i] - '0') % p, p);
  }
  return neg && x ? p - x : x;
}

inline Bytes packWords(const std::vector<u128>& v) {
  Bytes b(v.size() * AMPH_WORD_WIDTH);
  for (size_t i = 0; i < v.size(); ++i) storeLe(v[i], b.data() + 16 * i);
  return b;
}
inline std::vector<u128> unpackWords(const Bytes& b) {
  std::vector<u128> v(b.size() / 16);
  for (size_t i = 0; i < v.size(); ++i) v[i] = loadLe(b.data() + 16 * i);
  return v;
}

// MpSpdzIntegrationUtils.of(prime, r, rInv) on one GPU.
class Context {
 public:
  Context(u128 prime, u128 r, u128 rInv, int device = 0) : prime_(prime), r_(r), rInv_(rInv) {
    uint8_t p[16], rr[16], ri[16];
    storeLe(prime, p);
    storeLe(r, rr);
    storeLe(rInv, ri);
    check(amph_ctx_create(p, rr, ri, device, &h_));
  }
  ~Context() { amph_ctx_destroy(h_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  Context(Context&& o) noexcept : h_(o.h_), prime_(o.prime_), r_(o.r_), rInv_(o.rInv_) { o.h_ = nullptr; }
  amph_ctx* get() const { return h_; }
  u128 prime() const { return prime_; }
  u128 r() const { return r_; }
  u128 rInv() const { return rInv_; }

  Bytes toGfp(const std::vector<u128>& values) const {
    Bytes in = packWords(values), out(in.size());
    check(amph_to_gfp(h_, in.data(), values.size(), out.data(), 0, nullptr));
    return out;
  }
  std::vector<u128> fromGfp(const Bytes& words) const {
    Bytes out(words.size() / 16 * 16);
    check(amph_from_gfp(h_, words.data(), words.size() / 16, out.data(), 0, nullptr));
    return unpackWords(out);
  }

 private:
  amph_ctx* h_ = nullptr;
  u128 prime_, r_, rInv_;
};

class OutputDeliveryObject {
 public:
  OutputDeliveryObject(Bytes secretShares, Bytes rShares, Bytes vShares, Bytes wShares, Bytes uShares)
      : y_(std::move(secretShares)), r_(std::move(rShares)), v_(std::move(vShares)),
        w_(std::move(wShares)), u_(std::move(uShares)) {
    if (r_.size() != y_.size() || v_.size() != y_.size() || w_.size() != y_.size() ||
        u_.size() != y_.size())
      throw IllegalArgumentException("The provided shares must be of the same length");
  }
  const Bytes& getSecretShares() const { return y_; }
  const Bytes& getRShares() const { return r_; }
  const Bytes& getVShares() const { return v_; }
  const Bytes& getWShares() const { return w_; }
  const Bytes& getUShares() const { return u_; }
  amph_odo view() const {
    return amph_odo{y_.data(), r_.data(), v_.data(), w_.data(), u_.data(), y_.size()};
  }
  bool operator==(const OutputDeliveryObject& o) const {
    return y_ == o.y_ && r_ == o.r_ && v_ == o.v_ && w_ == o.w_ && u_ == o.u_;
  }

 private:
  Bytes y_, r_, v_, w_, u_;
};

namespace client {

class SecretShareUtil {
 public:
  static SecretShareUtil of(u128 prime, u128 r, u128 rInv, int device = 0) {
    return SecretShareUtil(Context(prime, r, rInv, device));
  }
  const Context& context() const { return ctx_; }
  u128 getPrime() const { return ctx_.prime(); }

  // maskInput :65-68 -> MaskedInputData (16 bytes)
  Bytes maskInput(u128 secret, u128 inputMask) const {
    Bytes s = packWords({secret % getPrime()}), m = packWords({inputMask % getPrime()}), out(16);
    check(amph_mask_words(ctx_.get(), s.data(), m.data(), 1, out.data(), 0, nullptr));
    return out;
  }

  // recombineObject :70-90 (parties of their own lengths: copyOfRange semantics,
  // ArrayIndexOutOfBoundsException for a word past a shorter party's end)
  std::vector<u128> recombineObject(const std::vector<Bytes>& shares) const {
    if (shares.empty()) return {};
    std::vector<const uint8_t*> ptrs;
    std::vector<size_t> lens;
    for (auto& s : shares) {
      ptrs.push_back(s.data());
      lens.push_back(s.size());
    }
    Bytes out(shares[0].size() / 16 * 16);
    check(amph_recombine_object(ctx_.get(), ptrs.data(), (int)ptrs.size(), lens.data(), out.data(), 0, nullptr));
    return unpackWords(out);
  }

  // verifySecrets :102-141 (Java argument order); all values canonical
  void verifySecrets(const std::vector<u128>& secrets, const std::vector<u128>& rs,
                     const std::vector<u128>& us, const std::vector<u128>& vs,
                     const std::vector<u128>& ws) const {
    const u128 p = getPrime();
    size_t pre = secrets.size();
    std::vector<u128> w2(ws), u2(us);
    for (size_t i = 0; i < secrets.size(); ++i)
      if (ws[i] >= p || us[i] >= p) {
        if (pre == secrets.size()) pre = i;
        w2[i] = u2[i] = 0;
      }
    Bytes y = packWords(reduce(secrets)), r = packWords(reduce(rs)), v = packWords(reduce(vs));
    Bytes w = packWords(w2), u = packWords(u2);
    int64_t ff = -1;
    const int st = amph_verify(ctx_.get(), y.data(), r.data(), u.data(), v.data(), w.data(),
                               secrets.size(), &ff, 0, nullptr);
    if (st != AMPH_OK && st != AMPH_E_VERIFY) check(st);
    size_t bad = st == AMPH_E_VERIFY ? (size_t)ff : secrets.size();
    if (pre < bad) bad = pre;
    if (bad < secrets.size())
      throw IntegrityVerificationException(
          message(secrets[bad], rs[bad], us[bad], vs[bad], ws[bad]));
  }

  std::string message(u128 y, u128 r, u128 u, u128 v, u128 w) const {
    uint8_t b[5][16];
    storeLe(y, b[0]);
    storeLe(r, b[1]);
    storeLe(u, b[2]);
    storeLe(v, b[3]);
    storeLe(w, b[4]);
    char buf[512];
    amph_verify_message(ctx_.get(), b[0], b[1], b[2], b[3], b[4], buf, sizeof buf);
    return buf;
  }

 private:
  explicit SecretShareUtil(Context&& c) : ctx_(std::move(c)) {}
  std::vector<u128> reduce(const std::vector<u128>& v) const {
    std::vector<u128> o(v);
    for (auto& x : o) x %= getPrime();
    return o;
  }
  Context ctx_;
};

// DefaultAmphoraClient.verifyOutputDeliveryObjects :476-505 (K_RV)
inline std::vector<u128> verifyOutputDeliveryObjects(const SecretShareUtil& util,
                                                     const std::vector<OutputDeliveryObject>& odos) {
  std::vector<amph_odo> v;
  for (auto& o : odos) v.push_back(o.view());
  const size_t W = odos.empty() ? 0 : odos[0].getSecretShares().size() / 16;
  Bytes out(W * 16);
  int64_t ff = -1;
  const int st = amph_recombine_verify(util.context().get(), v.data(), (int)v.size(), out.data(),
                                       &ff, 0, nullptr);
  if (st == AMPH_E_VERIFY) {
    std::vector<u128> f[5];
    for (int k = 0; k < 5; ++k) {
      std::vector<Bytes> sh;
      for (auto& o : odos) {
        const Bytes& src = k == 0 ? o.getSecretShares() : k == 1 ? o.getRShares() : k == 2 ? o.getVShares()
                         : k == 3 ? o.getWShares() : o.getUShares();
        sh.push_back(copyOfRange(src, 16 * ff, 16 * ff + 16));  // a ragged party's word: zero-padded
      }
      f[k] = util.recombineObject(sh);
    }
    throw IntegrityVerificationException(util.message(f[0][0], f[1][0], f[4][0], f[2][0], f[3][0]));
  }
  check(st);
  return unpackWords(out);
}

// DefaultAmphoraClient.createSecret arithmetic :150-160 (K_MASK): masked words
inline std::vector<Bytes> maskSecret(const SecretShareUtil& util, const std::vector<u128>& secret,
                                     const std::vector<OutputDeliveryObject>& maskOdos) {
  std::vector<amph_odo> v;
  for (auto& o : maskOdos) v.push_back(o.view());
  std::vector<u128> s(secret);
  for (auto& x : s) x %= util.getPrime();
  Bytes in = packWords(s), out(in.size());
  int64_t ff = -1;
  const int st = amph_mask_input(util.context().get(), v.data(), (int)v.size(), in.data(), s.size(),
                                 out.data(), &ff, 0, nullptr);
  if (st == AMPH_E_VERIFY) {
    verifyOutputDeliveryObjects(util, maskOdos);  // throws with the reference message
  }
  check(st);
  std::vector<Bytes> words;
  for (size_t i = 0; i < s.size(); ++i) words.emplace_back(out.begin() + 16 * i, out.begin() + 16 * i + 16);
  return words;
}

// The five base64 field strings of one party's VerifiableSecretShare /
// OutputDeliveryObject JSON body (secretShares, rShares, vShares, wShares,
// uShares), kept as text: the client hands them to the fused wire kernels.
struct OdoText {
  std::string f[5];
  // amph_odo_b64 carries ONE length for the five fields: unequal fields are
  // rejected here, before any copy reads them (OutputDeliveryObject.java:55-96).
  amph_odo_b64 view() const {
    for (int k = 1; k < 5; ++k)
      if (f[k].size() != f[0].size())
        throw IllegalArgumentException("The provided shares must be of the same length");
    return amph_odo_b64{f[0].data(), f[1].data(), f[2].data(), f[3].data(), f[4].data(), f[0].size()};
  }
};

inline size_t wordsOfBase64(const std::string& t) {
  const size_t pad = t.size() >= 2 ? (t[t.size() - 1] == '=') + (t[t.size() - 2] == '=') : 0;
  const size_t nb = t.size() / 4 * 3 - pad;
  if (t.size() % 4 || nb % 16) throw IllegalArgumentException("base64 field is not a whole number of words");
  return nb / 16;
}

// getSecret from the parties' response text (DefaultAmphoraClient.java:206-217
// incl. the base64 decode Jackson does per field): one launch of
// amph_recombine_verify_b64; a bad character -> AmphoraClientException.
inline std::vector<u128> verifyOutputDeliveryText(const SecretShareUtil& util,
                                                  const std::vector<OdoText>& odos) {
  std::vector<amph_odo_b64> v;
  for (auto& o : odos) v.push_back(o.view());
  const size_t W = odos.empty() ? 0 : wordsOfBase64(odos[0].f[0]);
  Bytes out(W * 16);
  int64_t ff = -1, bad = -1;
  const int st = amph_recombine_verify_b64(util.context().get(), v.data(), (int)v.size(), W, out.data(),
                                           &ff, &bad, 0, nullptr);
  if (st == AMPH_E_PARAM && bad >= 0) throw AmphoraClientException(amph_last_error());
  if (st == AMPH_E_VERIFY) {  // the reference message, from the decoded fields
    std::vector<OutputDeliveryObject> dec;
    for (auto& o : odos) {
      Bytes f[5];
      for (int k = 0; k < 5; ++k) {
        f[k].resize(3 * o.f[k].size() / 4);
        size_t nb = 0;
        int64_t b2 = -1;
        check(amph_base64_decode(util.context().get(), o.f[k].data(), o.f[k].size(), f[k].data(), &nb, &b2, 0,
                                 nullptr));
        f[k].resize(nb);
      }
      dec.emplace_back(f[0], f[1], f[2], f[3], f[4]);
    }
    verifyOutputDeliveryObjects(util, dec);  // throws IntegrityVerificationException
  }
  check(st);
  return unpackWords(out);
}

// createSecret from the parties' /input-masks response text: verify + mask +
// the MaskedInputData base64 records (24 characters per word), one launch of
// amph_mask_input_b64.
inline std::vector<std::string> maskSecretText(const SecretShareUtil& util, const std::vector<u128>& secret,
                                               const std::vector<OdoText>& maskOdos) {
  std::vector<amph_odo_b64> v;
  for (auto& o : maskOdos) v.push_back(o.view());
  const size_t W = maskOdos.empty() ? 0 : wordsOfBase64(maskOdos[0].f[0]);
  std::vector<u128> s(secret);
  for (auto& x : s) x %= util.getPrime();
  Bytes in = packWords(s);
  std::string rec(24 * s.size(), '\0');
  int64_t ff = -1, bad = -1;
  const int st = amph_mask_input_b64(util.context().get(), v.data(), (int)v.size(), W, in.data(), s.size(),
                                     nullptr, &rec[0], &ff, &bad, 0, nullptr);
  if (st == AMPH_E_PARAM && bad >= 0) throw AmphoraClientException(amph_last_error());
  if (st == AMPH_E_VERIFY) verifyOutputDeliveryText(util, maskOdos);  // throws with the message
  // more secret words than masks: the ABI has verified every mask first
  // (DefaultAmphoraClient.java:153 before :155-157), so this is an honest set
  if (st == AMPH_E_LEN && s.size() > W)
    throw std::out_of_range("Index " + std::to_string(W) + " out of bounds for length " + std::to_string(W));
  check(st);
  std::vector<std::string> out;
  for (size_t i = 0; i < s.size(); ++i) out.push_back(rec.substr(24 * i, 24));
  return out;
}

}  // namespace client

namespace service {

// One request's Output Delivery with the triples, diffs and ODO fields kept on
// the GPU between the steps (amph_party_*): begin -> text() -> partner(slot,
// ...) for every partner -> finish().
class PartySession {
 public:
  PartySession(const Context& ctx, const Bytes& shareData, size_t stride, const Bytes& maskTuples,
               const Bytes& triples, int nParties)
      : words_(shareData.size() / stride), y_(16 * words_), r_(16 * words_), v_(16 * words_) {
    check(amph_party_begin(ctx.get(), shareData.data(), stride, maskTuples.data(), triples.data(), words_,
                           nParties, y_.data(), r_.data(), v_.data(), &p_));
  }
  PartySession(const PartySession&) = delete;
  PartySession& operator=(const PartySession&) = delete;
  ~PartySession() { amph_party_free(p_); }

  // this party's interimValues array (the FactorPair JSON Jackson writes)
  std::string text() const {
    std::string t(amph_party_text_len(p_), '\0');
    check(amph_party_text(p_, &t[0], t.size()));
    return t;
  }
  // a partner's interimValues array; IllegalArgumentException if malformed
  void partner(int slot, const char* text, size_t len) {
    int64_t bad = -1;
    const int st = amph_party_partner(p_, slot, text, len, &bad);
    if ((st == AMPH_E_PARAM || st == AMPH_E_LEN) && bad >= 0) throw IllegalArgumentException(amph_last_error());
    check(st);
  }
  OutputDeliveryObject finish(bool isPlayer0) {
    Bytes w(16 * words_), u(16 * words_);
    check(amph_party_finish(p_, isPlayer0, w.data(), u.data()));
    return OutputDeliveryObject(std::move(y_), std::move(r_), std::move(v_), std::move(w), std::move(u));
  }

 private:
  size_t words_;
  Bytes y_, r_, v_;
  amph_party* p_ = nullptr;
};

class SecretShareUtil {
 public:
  explicit SecretShareUtil(const Context& ctx) : ctx_(ctx) {}
  // convertToSecretShare :58-81; maskedInput: 16-B words, inputMasks: 32-B
  // tuples (value || mac of share 0).  Returns SecretShare.data (32 B/word).
  Bytes convertToSecretShare(const std::vector<Bytes>& maskedInput, const std::string& macKey,
                             const Bytes& inputMasks, bool useZeroInputAsData) const {
    if (maskedInput.size() != inputMasks.size() / 32)
      throw IllegalArgumentException("Received more input data than available inputMasks.");
    Bytes m;
    for (auto& w : maskedInput) m.insert(m.end(), w.begin(), w.end());
    uint8_t key[16];
    storeLe(fromDecimal(macKey, ctx_.prime()), key);
    Bytes out(maskedInput.size() * 32);
    check(amph_convert_share(ctx_.get(), m.data(), inputMasks.data(), maskedInput.size(), key,
                             useZeroInputAsData, out.data(), 0, nullptr));
    return out;
  }

 private:
  const Context& ctx_;
};

}  // namespace service

// java.util.UUID.nameUUIDFromBytes: MD5 (RFC 1321) with the version-3 and
// IETF-variant bits set, rendered 8-4-4-4-12 in lower-case hex.
inline std::array<uint8_t, 16> md5(const uint8_t* msg, size_t len) {
  uint32_t K[64];
  for (int i = 0; i < 64; ++i) K[i] = (uint32_t)(std::fabs(std::sin((double)(i + 1))) * 4294967296.0);
  static const int S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  Bytes m(msg, msg + len);
  m.push_back(0x80);
  while (m.size() % 64 != 56) m.push_back(0);
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) m.push_back((uint8_t)(bits >> (8 * i)));
  for (size_t off = 0; off < m.size(); off += 64) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)m[off + 4 * i] | ((uint32_t)m[off + 4 * i + 1] << 8) |
             ((uint32_t)m[off + 4 * i + 2] << 16) | ((uint32_t)m[off + 4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; ++i) {
      uint32_t f;
      int g;
      if (i < 16) { f = (b & c) | (~b & d); g = i; }
      else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) % 16; }
      else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) % 16; }
      else { f = c ^ (b | ~d); g = (7 * i) % 16; }
      const uint32_t t = d;
      d = c;
      c = b;
      const uint32_t x = a + f + K[i] + w[g];
      const int r = S[(i / 16) * 4 + i % 4];
      b = b + ((x << r) | (x >> (32 - r)));
      a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  }
  std::array<uint8_t, 16> out;
  for (int i = 0; i < 16; ++i) out[i] = (uint8_t)(h[i / 4] >> (8 * (i % 4)));
  return out;
}

inline std::string nameUUIDFromBytes(const std::string& name) {
  auto d = md5(reinterpret_cast<const uint8_t*>(name.data()), name.size());
  d[6] = (uint8_t)((d[6] & 0x0f) | 0x30);
  d[8] = (uint8_t)((d[8] & 0x3f) | 0x80);
  static const char* hex = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < 16; ++i) {
    if (i == 4 || i == 6 || i == 8 || i == 10) s += '-';
    s += hex[d[i] >> 4];
    s += hex[d[i] & 15];
  }
  return s;
}

namespace wire {

// base64 as Jackson writes byte[] (MIME_NO_LINEFEEDS), on the GPU.
inline std::string base64Encode(const Context& ctx, const Bytes& data) {
  std::string out(4 * ((data.size() + 2) / 3), '\0');
  check(amph_base64_encode(ctx.get(), data.data(), data.size(), &out[0], 0, nullptr));
  return out;
}

inline Bytes base64Decode(const Context& ctx, const std::string& text) {
  Bytes out(3 * text.size() / 4);
  size_t n = 0;
  int64_t bad = -1;
  const int st = amph_base64_decode(ctx.get(), text.data(), text.size(), out.data(), &n, &bad, 0, nullptr);
  if (st == AMPH_E_PARAM || st == AMPH_E_LEN) throw IllegalArgumentException(amph_last_error());
  check(st);
  out.resize(n);
  return out;
}

inline std::string exchangeBody(const std::string& operationId, int playerId, const std::string& interimValues);

// Signed Beaver diffs in amph_odo_pre's layout: 2 values per pair.
struct Diffs {
  Bytes mag;  // 32 B per pair (d, e magnitudes, LE16)
  Bytes neg;  // 2 sign bytes per pair
  size_t pairs() const { return neg.size() / 2; }
};

// MultiplicationExchangeObject -> its JSON body (byte-identical to Jackson's
// default compact serialisation).
inline std::string exchangeToJson(const Context& ctx, const std::string& operationId, int playerId,
                                  const Diffs& d) {
  std::string arr(amph_exchange_max_chars(d.pairs()), '\0');
  uint64_t n = 0;
  check(amph_exchange_encode(ctx.get(), d.mag.data(), d.neg.data(), d.pairs(), &arr[0], arr.size(), &n,
                             0, nullptr));
  arr.resize(n);
  return exchangeBody(operationId, playerId, arr);
}

// A MultiplicationExchangeObject JSON body: its operationId and the span
// [lb, rb] of its interimValues array.
struct ExchangeSpan {
  std::string operationId;
  size_t lb, rb;
};

inline ExchangeSpan exchangeSpan(const std::string& body) {
  const size_t k = body.find("\"interimValues\"");
  const size_t lb = k == std::string::npos ? k : body.find('[', k);
  const size_t rb = body.rfind(']');
  if (lb == std::string::npos || rb == std::string::npos || rb < lb)
    throw IllegalArgumentException("interimValues is marked non-null but is null");
  std::string op;
  const size_t o = body.find("\"operationId\"");
  if (o != std::string::npos) {
    const size_t q0 = body.find('"', body.find(':', o) + 1);
    const size_t q1 = q0 == std::string::npos ? q0 : body.find('"', q0 + 1);
    if (q1 != std::string::npos) op = body.substr(q0 + 1, q1 - q0 - 1);
  }
  if (op.empty()) throw IllegalArgumentException("operationId is marked non-null but is null");
  return {op, lb, rb};
}

inline std::string exchangeBody(const std::string& operationId, int playerId, const std::string& interimValues) {
  return "{\"operationId\":\"" + operationId + "\",\"playerId\":" + std::to_string(playerId) +
         ",\"interimValues\":" + interimValues + "}";
}

// JSON body -> (operationId, diffs); the interimValues array is parsed on the GPU.
inline std::pair<std::string, Diffs> exchangeFromJson(const Context& ctx, const std::string& body,
                                                      size_t pairs) {
  const ExchangeSpan sp = exchangeSpan(body);
  Diffs d{Bytes(32 * pairs), Bytes(2 * pairs)};
  int64_t bad = -1;
  const int st = amph_exchange_decode(ctx.get(), body.data() + sp.lb, sp.rb + 1 - sp.lb, pairs, d.mag.data(),
                                      d.neg.data(), &bad, 0, nullptr);
  if (st == AMPH_E_PARAM || st == AMPH_E_LEN) throw IllegalArgumentException(amph_last_error());
  check(st);
  return {sp.operationId, std::move(d)};
}

}  // namespace wire

namespace service {

// OutputDeliveryService.computeOutputDeliveryObject (:75-161) with Castor and
// the inter-VCP open injected: tuples(requestId, tupleType, count) returns
// the tuple stream ("INPUT_MASK_GFP": 32 B each, "MULTIPLICATION_TRIPLE_GFP":
// 96 B each); exchange(ownJson) returns the partners' JSON bodies.
class OutputDeliveryService {
 public:
  using TupleSource = std::function<Bytes(const std::string&, const std::string&, size_t)>;
  using Exchange = std::function<std::vector<std::string>(const std::string&)>;

  // sessionParties > 0: run each request as a PartySession of that many parties
  // (same bodies and results; the triples and diffs stay on the GPU)
  OutputDeliveryService(const Context& ctx, int playerId, TupleSource tuples, Exchange exchange,
                        int sessionParties = 0)
      : ctx_(ctx), playerId_(playerId), tuples_(std::move(tuples)), exchange_(std::move(exchange)),
        sessionParties_(sessionParties) {}

  // shareData: SecretShare.data (stride 32, MACs stripped) or raw words (stride 16)
  OutputDeliveryObject computeOutputDeliveryObject(const Bytes& shareData, size_t stride,
                                                   const std::string& requestId) {
    const size_t W = shareData.size() / stride;
    const Bytes masks = download(requestId, "INPUT_MASK_GFP", 2 * W, 32);
    const std::string op = nameUUIDFromBytes(requestId + "_" + std::to_string(2 * W));  // :140-141
    const Bytes triples = download(op, "MULTIPLICATION_TRIPLE_GFP", 2 * W, 96);
    if (sessionParties_ > 0) return computeInSession(shareData, stride, masks, triples, op);
    Bytes y(16 * W), r(16 * W), v(16 * W);
    wire::Diffs own{Bytes(64 * W), Bytes(4 * W)};
    check(amph_odo_pre(ctx_.get(), shareData.data(), stride, masks.data(), triples.data(), W, y.data(),
                       r.data(), v.data(), own.mag.data(), own.neg.data(), 0, nullptr));
    lastExchange_ = wire::exchangeToJson(ctx_, op, playerId_, own);
    std::vector<wire::Diffs> partners;
    try {
      for (const std::string& body : exchange_(lastExchange_)) {
        auto pd = wire::exchangeFromJson(ctx_, body, 2 * W);
        if (pd.first != op) throw IllegalArgumentException("operation id mismatch");
        partners.push_back(std::move(pd.second));
      }
    } catch (const std::exception&) {  // the cause stays attached (std::rethrow_if_nested), as Java chains it
      std::throw_with_nested(AmphoraServiceException("Failed to open values for operation #" + op));
    }
    std::vector<const uint8_t*> mags{own.mag.data()}, negs{own.neg.data()};
    for (auto& pd : partners) {
      mags.push_back(pd.mag.data());
      negs.push_back(pd.neg.data());
    }
    Bytes w(16 * W), u(16 * W);  // recombineDiffs + multiplySharedSecrets, fused
    check(amph_open_post(ctx_.get(), mags.data(), negs.data(), (int)mags.size(), triples.data(), W,
                         playerId_ == 0, w.data(), u.data(), 0, nullptr));
    return OutputDeliveryObject(std::move(y), std::move(r), std::move(v), std::move(w), std::move(u));
  }

  const std::string& lastExchangeObject() const { return lastExchange_; }

 private:
  OutputDeliveryObject computeInSession(const Bytes& shareData, size_t stride, const Bytes& masks,
                                        const Bytes& triples, const std::string& op) {
    PartySession s(ctx_, shareData, stride, masks, triples, sessionParties_);
    lastExchange_ = wire::exchangeBody(op, playerId_, s.text());
    try {
      const std::vector<std::string> bodies = exchange_(lastExchange_);
      if ((int)bodies.size() != sessionParties_ - 1) throw IllegalArgumentException("partner count mismatch");
      int slot = 1;
      for (const std::string& body : bodies) {
        const wire::ExchangeSpan sp = wire::exchangeSpan(body);
        if (sp.operationId != op) throw IllegalArgumentException("operation id mismatch");
        s.partner(slot++, body.data() + sp.lb, sp.rb + 1 - sp.lb);
      }
    } catch (const std::exception&) {
      std::throw_with_nested(AmphoraServiceException("Failed to open values for operation #" + op));
    }
    return s.finish(playerId_ == 0);
  }

  Bytes download(const std::string& id, const char* type, size_t count, size_t width) {
    Bytes b;
    try {
      b = tuples_(id, type, count);
    } catch (const std::exception&) {  // :103-107, :178-185
      std::throw_with_nested(AmphoraServiceException("Failed to retrieve the required Tuples form Castor"));
    }
    if (b.size() != count * width)
      throw AmphoraServiceException("Failed to retrieve the required Tuples form Castor");
    return b;
  }

  const Context& ctx_;
  int playerId_;
  TupleSource tuples_;
  Exchange exchange_;
  int sessionParties_;
  std::string lastExchange_;
};

}  // namespace service
}  // namespace amphora

#endif  // AMPHORA_HPP_
