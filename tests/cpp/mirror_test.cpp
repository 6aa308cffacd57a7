// C++ host-mirror test (include/amphora.hpp).  Mode "cpu": host-only checks
// (context validation, decimal parsing, message format).  Mode "gpu": the
// reference's KATs and a round trip through the GPU kernels.
//   KAT-1  amphora-service/.../calculation/SecretShareUtilTest.java:68-107
//   KAT-3  amphora-java-client/.../SecretShareUtilTest.java:30-85
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

#include "amphora.hpp"

using namespace amphora;

static int failures = 0;
#define EXPECT(c)                                                     \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

static const u128 P = fromDecimal("198766463529478683931867765928436695041", ~(u128)0);
static const u128 R = fromDecimal("141515903391459779531506841503331516415", ~(u128)0);
static const u128 RI = fromDecimal("133854242216446749056083838363708373830", ~(u128)0);

static void cpu_tests() {
  Context c(P, R, RI);
  EXPECT(toDecimal(P) == "198766463529478683931867765928436695041");
  EXPECT(fromDecimal("-1", P) == P - 1);
  EXPECT(fromDecimal("-33717010807885571165607137982809795379", P) ==
         P - fromDecimal("33717010807885571165607137982809795379", P));
  bool threw = false;
  try {
    Context bad(P, R + 1, RI);
  } catch (const NativeError& e) {
    threw = e.status == AMPH_E_PARAM;
  }
  EXPECT(threw);
  auto util = client::SecretShareUtil::of(P, R, RI);
  EXPECT(util.message(5, 7, 21, 3, 36) ==
         "Verification of secret has failed:\n\t36 = 5 * 7   &&   21 = 3 * 7\n\t36 = 35   &&   21 = 21");
  threw = false;
  try {
    OutputDeliveryObject o(Bytes(16), Bytes(16), Bytes(32), Bytes(16), Bytes(16));
  } catch (const IllegalArgumentException& e) {
    threw = std::string(e.what()) == "The provided shares must be of the same length";
  }
  EXPECT(threw);
  // java.util.UUID.nameUUIDFromBytes (OutputDeliveryServiceTest.java operation id)
  auto d0 = md5(nullptr, 0);
  EXPECT(d0[0] == 0xd4 && d0[1] == 0x1d && d0[15] == 0x7e);  // md5("") = d41d8c...f8427e
  EXPECT(nameUUIDFromBytes("70297fd4-d412-4dbb-af05-6818fe0e687a_4") == "8065e700-9f48-36ba-ae8c-f881b28a28ef");
}

// KAT-2 (OutputDeliveryServiceTest.java:64-175) through the C++ service, the
// open carried as MultiplicationExchangeObject JSON bodies.
static void kat2_service(const Context& c) {
  const std::vector<u128> secrets = {90, 142}, masks = {87, 111, 412, 313};
  const u128 tri[4][3] = {{80, 62, 3719}, {72, 63, 32521}, {141, 264, 56212}, {19, 35, 612}};
  auto g = [&](u128 x) { return c.toGfp({x}); };
  auto cat = [](Bytes& a, const Bytes& b) { a.insert(a.end(), b.begin(), b.end()); };
  Bytes share, maskTuples, triples;
  for (u128 s : secrets) { cat(share, g(s)); cat(share, g(0)); }
  for (u128 m : masks) { cat(maskTuples, g(m)); cat(maskTuples, g(0)); }
  for (auto& t : tri)
    for (int k = 0; k < 3; ++k) { cat(triples, g(t[k])); cat(triples, g(0)); }
  const std::string req = "70297fd4-d412-4dbb-af05-6818fe0e687a", op = "8065e700-9f48-36ba-ae8c-f881b28a28ef";
  const std::string own = "{\"operationId\":\"" + op + "\",\"playerId\":0,\"interimValues\":"
                          "[{\"a\":10,\"b\":25},{\"a\":39,\"b\":24},{\"a\":1,\"b\":148},{\"a\":294,\"b\":377}]}";
  const std::string partner = "{\"operationId\":\"" + op + "\",\"playerId\":1,\"interimValues\":"
                              "[{\"a\":4,\"b\":63},{\"a\":175,\"b\":136},{\"a\":5,\"b\":106},{\"a\":2,\"b\":27}]}";
  for (int sessionParties : {0, 2}) {  // per-call path, then as a device-resident party session
    bool ownOk = false;
    service::OutputDeliveryService svc(
        c, 0,
        [&](const std::string& id, const std::string& type, size_t count) {
          EXPECT(count == 4);
          if (type == "INPUT_MASK_GFP") { EXPECT(id == req); return maskTuples; }
          EXPECT(type == "MULTIPLICATION_TRIPLE_GFP" && id == op);
          return triples;
        },
        [&](const std::string& body) {
          ownOk = body == own;
          return std::vector<std::string>{partner};
        },
        sessionParties);
    OutputDeliveryObject odo = svc.computeOutputDeliveryObject(share, 32, req);
    EXPECT(ownOk);
    EXPECT(odo == OutputDeliveryObject(c.toGfp(secrets), c.toGfp({87, 412}), c.toGfp({111, 313}),
                                       c.toGfp({12859, 95134}), c.toGfp({91763, 138232})));
  }
  {  // a malformed partner body in a session: the reference's open failure, the cause nested
    service::OutputDeliveryService svc(
        c, 0, [&](const std::string&, const std::string& type, size_t) {
          return type == "INPUT_MASK_GFP" ? maskTuples : triples;
        },
        [&](const std::string&) {
          std::string bad = partner;
          bad[bad.find("175")] = 'x';
          return std::vector<std::string>{bad};
        },
        2);
    bool threw = false;
    try {
      svc.computeOutputDeliveryObject(share, 32, req);
    } catch (const AmphoraServiceException& e) {
      threw = std::string(e.what()) == "Failed to open values for operation #" + op;
    }
    EXPECT(threw);
  }
  bool threw = false;
  service::OutputDeliveryService broken(
      c, 0, [&](const std::string&, const std::string&, size_t) -> Bytes { throw std::runtime_error("x"); },
      [&](const std::string&) { return std::vector<std::string>{}; });
  try {
    broken.computeOutputDeliveryObject(share, 32, req);
  } catch (const AmphoraServiceException& e) {
    threw = std::string(e.what()) == "Failed to retrieve the required Tuples form Castor";
  }
  EXPECT(threw);
  // base64 as Jackson writes byte[] (VerifiableSecretTest.java)
  const std::string b = wire::base64Encode(c, Bytes{'s', 'S', 'h', 'a', 'r', 'e', 's'});
  EXPECT(b == "c1NoYXJlcw==");
  EXPECT(wire::base64Decode(c, b) == (Bytes{'s', 'S', 'h', 'a', 'r', 'e', 's'}));
}

static void gpu_tests() {
  auto util = client::SecretShareUtil::of(P, R, RI);
  const Context& c = util.context();
  // KAT-1
  service::SecretShareUtil ssu(c);
  auto v = [&](const char* d) { return fromDecimal(d, P); };
  const u128 key = v("-33717010807885571165607137982809795379");
  Bytes masked = c.toGfp({v("37371993412255263319479925008425883363"), 0});
  Bytes masks = c.toGfp({v("-82730997414791468496799367418496881908"), v("-60557275363670854182192939229091375859"),
                         v("45359004002536205186084333850157344582"), v("-48604663536222227589564560476962533035")});
  Bytes expected = c.toGfp({v("-45359004002536205177319442410070998545"), v("-170814686092998134911558977038957876158"),
                            v("45359004002536205186084333850157344582"), v("-48604663536222227589564560476962533035")});
  std::vector<Bytes> mi = {Bytes(masked.begin(), masked.begin() + 16), Bytes(masked.begin() + 16, masked.end())};
  EXPECT(ssu.convertToSecretShare(mi, toDecimal(key), masks, false) == expected);
  bool threw = false;
  try {
    ssu.convertToSecretShare({Bytes(16)}, "", Bytes(), false);
  } catch (const IllegalArgumentException& e) {
    threw = std::string(e.what()) == "Received more input data than available inputMasks.";
  }
  EXPECT(threw);
  // KAT-3 structure: w = s r, u = v r unreduced (< p) pass; w[last] -= 10 fails
  std::mt19937_64 rng(42);
  auto nl = [&]() { return (u128)(rng() >> 1); };
  std::vector<u128> s, r, vv, w, u;
  for (int i = 0; i < 5; ++i) {
    s.push_back(nl()); r.push_back(nl()); vv.push_back(nl());
    w.push_back(s[i] * r[i]); u.push_back(vv[i] * r[i]);
  }
  util.verifySecrets(s, r, u, vv, w);
  w[4] -= 10;
  threw = false;
  try {
    util.verifySecrets(s, r, u, vv, w);
  } catch (const IntegrityVerificationException& e) {
    threw = std::string(e.what()).rfind("Verification of secret has failed", 0) == 0;
  }
  EXPECT(threw);
  // round trip: 2-party ODOs of secrets, recombine + verify recovers them
  const size_t W = 777;
  std::vector<u128> sec(W), share0[5], share1[5];
  for (size_t i = 0; i < W; ++i) sec[i] = ((u128)rng() << 64 | rng()) % P;
  std::vector<u128> rr(W), vr(W);
  for (size_t i = 0; i < W; ++i) { rr[i] = ((u128)rng() << 64 | rng()) % P; vr[i] = rng(); }
  // test data: w = s r mod p by a host double-and-add ladder (independent of
  // the kernels' Montgomery products)
  auto mulmod = [&](u128 a, u128 b) {
    u128 acc = 0;
    for (int bit = 127; bit >= 0; --bit) {
      acc = addMod(acc, acc, P);
      if ((b >> bit) & 1) acc = addMod(acc, a % P, P);
    }
    return acc;
  };
  std::vector<u128> vals[5];
  for (size_t i = 0; i < W; ++i) {
    vals[0].push_back(sec[i]); vals[1].push_back(rr[i]); vals[2].push_back(vr[i] % P);
    vals[3].push_back(mulmod(sec[i], rr[i])); vals[4].push_back(mulmod(vr[i] % P, rr[i]));
  }
  Bytes parts[2][5];
  for (int k = 0; k < 5; ++k) {
    std::vector<u128> a(W), b(W);
    for (size_t i = 0; i < W; ++i) {
      a[i] = ((u128)rng() << 64 | rng()) % P;
      b[i] = vals[k][i] >= a[i] ? vals[k][i] - a[i] : vals[k][i] + (P - a[i]);
    }
    parts[0][k] = c.toGfp(a);
    parts[1][k] = c.toGfp(b);
  }
  std::vector<OutputDeliveryObject> odos;
  for (int j = 0; j < 2; ++j)
    odos.emplace_back(parts[j][0], parts[j][1], parts[j][2], parts[j][3], parts[j][4]);
  EXPECT(client::verifyOutputDeliveryObjects(util, odos) == sec);
  // masking with these as Input Mask ODOs: masked + mask == secret
  std::vector<u128> secrets(W);
  for (auto& x : secrets) x = rng();
  auto maskedWords = client::maskSecret(util, secrets, odos);
  for (size_t i = 0; i < W; i += 97) {
    const u128 mv = c.fromGfp(maskedWords[i])[0];
    EXPECT(addMod(mv, sec[i], P) == secrets[i] % P);
  }
  // tamper party 1's w share of word 5 -> IntegrityVerificationException
  Bytes wt = parts[1][3];
  wt[16 * 5] ^= 1;
  std::vector<OutputDeliveryObject> bad = {odos[0], OutputDeliveryObject(parts[1][0], parts[1][1], parts[1][2], wt, parts[1][4])};
  threw = false;
  try {
    client::verifyOutputDeliveryObjects(util, bad);
  } catch (const IntegrityVerificationException&) {
    threw = true;
  }
  EXPECT(threw);
  // the same round trip from the response text (fused wire kernels)
  std::vector<client::OdoText> texts(2);
  for (int j = 0; j < 2; ++j)
    for (int k = 0; k < 5; ++k) texts[j].f[k] = wire::base64Encode(c, parts[j][k]);
  for (int rep = 0; rep < 16; ++rep) {  // repeated one-shot host calls (fresh staging each time)
    EXPECT(client::verifyOutputDeliveryText(util, texts) == sec);
    EXPECT(client::maskSecretText(util, secrets, texts).size() == W);
  }
  auto records = client::maskSecretText(util, secrets, texts);
  EXPECT(records.size() == W);
  for (size_t i = 0; i < W; i += 97) EXPECT(records[i] == wire::base64Encode(c, maskedWords[i]));
  auto tamperedText = texts;
  tamperedText[1].f[3] = wire::base64Encode(c, wt);
  threw = false;
  try {
    client::verifyOutputDeliveryText(util, tamperedText);
  } catch (const IntegrityVerificationException& e) {
    threw = std::string(e.what()).rfind("Verification of secret has failed", 0) == 0;
  }
  EXPECT(threw);
  auto badChar = texts;
  badChar[0].f[2][100] = '*';
  threw = false;
  try {
    client::verifyOutputDeliveryText(util, badChar);
  } catch (const AmphoraClientException& e) {
    threw = std::string(e.what()).find("index 100 of party 0's vShares") != std::string::npos;
  }
  EXPECT(threw);
  // one party's field shorter than its secretShares: rejected before any
  // copy reads past it (host heap over-read otherwise)
  auto shortField = texts;
  shortField[1].f[2].resize(shortField[1].f[2].size() - 4);
  for (int fn = 0; fn < 2; ++fn) {
    threw = false;
    try {
      if (fn == 0) client::verifyOutputDeliveryText(util, shortField);
      else client::maskSecretText(util, secrets, shortField);
    } catch (const IllegalArgumentException& e) {
      threw = std::string(e.what()) == "The provided shares must be of the same length";
    }
    EXPECT(threw);
  }
  // more secret words than masks: a tampered mask set fails verification
  // first (DefaultAmphoraClient.java:153), an honest one the index check
  std::vector<u128> longer(secrets);
  longer.push_back(1);
  threw = false;
  try {
    client::maskSecretText(util, longer, tamperedText);
  } catch (const IntegrityVerificationException&) {
    threw = true;
  }
  EXPECT(threw);
  threw = false;
  try {
    client::maskSecretText(util, longer, texts);
  } catch (const std::out_of_range&) {
    threw = true;
  }
  EXPECT(threw);
}

// recombineObject's ragged partner arrays (SecretShareUtil.java:75,87-88) through
// the mirror: longer -> cut; 8 bytes short -> last word zero-padded, MAC failure
// at W-1 with the reference's message; two words short -> ArrayIndexOutOfBounds.
static void ragged_tests(const client::SecretShareUtil& util) {
  const Context& c = util.context();
  const size_t W = 6;
  std::vector<u128> ys, rs, vs;
  std::mt19937_64 rng(7);
  for (size_t i = 0; i < W; ++i) {  // 63-bit values: the products stay below p
    ys.push_back((u128)(rng() >> 1));
    rs.push_back((u128)(rng() >> 1));
    vs.push_back((u128)(rng() >> 1));
  }
  auto prod = [&](const std::vector<u128>& a, const std::vector<u128>& b) {
    std::vector<u128> o;
    for (size_t i = 0; i < a.size(); ++i) o.push_back(a[i] * b[i]);
    return o;
  };
  const std::vector<u128> ws = prod(ys, rs), us = prod(vs, rs);
  // honest 2-party shares: party 1 random, party 0 the difference mod p
  auto subMod = [](u128 a, u128 b) { return a >= b ? a - b : a + (P - b); };
  auto share1 = [&]() {
    std::vector<u128> o;
    for (size_t i = 0; i < W; ++i) o.push_back((((u128)rng() << 64) | rng()) % P);
    return o;
  };
  auto minus = [&](const std::vector<u128>& a, const std::vector<u128>& b) {
    std::vector<u128> o;
    for (size_t i = 0; i < a.size(); ++i) o.push_back(subMod(a[i], b[i]));
    return o;
  };
  const std::vector<u128> y1 = share1(), r1 = share1(), v1 = share1(), w1 = share1(), u1 = share1();
  auto odo = [&](const std::vector<u128>& y, const std::vector<u128>& r, const std::vector<u128>& v,
                 const std::vector<u128>& w, const std::vector<u128>& u, long delta) {
    Bytes f[5] = {c.toGfp(y), c.toGfp(r), c.toGfp(v), c.toGfp(w), c.toGfp(u)};
    for (auto& b : f) b.resize((size_t)((long)b.size() + delta), 0x5A);
    return OutputDeliveryObject(f[0], f[1], f[2], f[3], f[4]);
  };
  const OutputDeliveryObject p0 = odo(minus(ys, y1), minus(rs, r1), minus(vs, v1), minus(ws, w1), minus(us, u1), 0);
  auto p1 = [&](long delta) { return odo(y1, r1, v1, w1, u1, delta); };
  EXPECT(client::verifyOutputDeliveryObjects(util, {p0, p1(0)}) == ys);
  EXPECT(client::verifyOutputDeliveryObjects(util, {p0, p1(40)}) == ys);  // longer: cut
  bool threw = false;
  try {  // 8 bytes short: the last word zero-padded, its MAC check fails
    client::verifyOutputDeliveryObjects(util, {p0, p1(-8)});
  } catch (const IntegrityVerificationException& e) {
    threw = std::string(e.what()).rfind("Verification of secret has failed:", 0) == 0;
  }
  EXPECT(threw);
  threw = false;
  try {
    client::verifyOutputDeliveryObjects(util, {p0, p1(-32)});
  } catch (const ArrayIndexOutOfBoundsException&) {
    threw = true;
  }
  EXPECT(threw);
  Bytes a = c.toGfp(ys), b(16 * W - 8, 0);
  EXPECT(util.recombineObject({a, b}) == ys);  // zero shares, zero padding: the values themselves
  threw = false;
  try {
    util.recombineObject({a, Bytes(16 * W - 17, 0)});
  } catch (const ArrayIndexOutOfBoundsException&) {
    threw = true;
  }
  EXPECT(threw);
  EXPECT(copyOfRange(Bytes{1, 2, 3}, 2, 6) == (Bytes{3, 0, 0, 0}));
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  try {
    cpu_tests();
    if (mode == "gpu") {
      gpu_tests();
      ragged_tests(client::SecretShareUtil::of(P, R, RI));
      Context c(P, R, RI);
      kat2_service(c);
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 2;
  }
  std::printf("%s: %d failures\n", mode.c_str(), failures);
  return failures ? 1 : 0;
}
