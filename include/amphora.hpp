// C++17 host-side mirror of the reference's Java interface over the C ABI
// (include/amphora.h).  Header-only; link against libamphora_hip.so.
//
//   amphora::client::SecretShareUtil       <- amphora-java-client/.../client/SecretShareUtil.java:33-157
//   amphora::client::verifyOutputDeliveryObjects / maskSecret
//                                          <- DefaultAmphoraClient.java:150-160,476-505
//   amphora::service::SecretShareUtil      <- amphora-service/.../calculation/SecretShareUtil.java:30-107
//   amphora::service::OutputDeliveryService<- amphora-service/.../calculation/OutputDeliveryService.java:57-286
//   amphora::OutputDeliveryObject          <- amphora-common/.../OutputDeliveryObject.java:55-106
//
// Java BigIntegers become `amphora::u128` canonical integers (callers reduce
// arbitrary-size values mod p before constructing them; `fromDecimal` does
// that for decimal strings like the MAC key property).  Exceptions carry the
// reference's messages.  Every word of arithmetic runs on the GPU.
#ifndef AMPHORA_HPP_
#define AMPHORA_HPP_

#include <cstdint>
#include <cstring>
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
struct NativeError : std::runtime_error {
  int status;
  NativeError(int st, const std::string& m) : std::runtime_error(m), status(st) {}
};

inline void check(int st) {
  if (st != AMPH_OK) throw NativeError(st, std::string(amph_strerror(st)) + ": " + amph_last_error());
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

  // recombineObject :70-90
  std::vector<u128> recombineObject(const std::vector<Bytes>& shares) const {
    if (shares.empty()) return {};
    std::vector<const uint8_t*> ptrs;
    for (auto& s : shares) {
      if (s.size() / 16 < shares[0].size() / 16) throw std::out_of_range("share arrays shorter than the first");
      ptrs.push_back(s.data());
    }
    const size_t nb = shares[0].size() / 16 * 16;
    Bytes out(nb);
    check(amph_recombine(ctx_.get(), ptrs.data(), (int)ptrs.size(), nb, out.data(), 0, nullptr));
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
        sh.emplace_back(src.begin() + 16 * ff, src.begin() + 16 * ff + 16);
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

}  // namespace client

namespace service {

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
}  // namespace amphora

#endif  // AMPHORA_HPP_
