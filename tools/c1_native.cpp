// BASELINE config C1 in native host code (tool): a W-word secret uploaded
// (createSecret) and downloaded (getSecret) through the C++ mirror of
// DefaultAmphoraClient / amphora-service (include/amphora.hpp) against two
// in-process parties.  The inter-VCP open travels as MultiplicationExchange-
// Object JSON bodies between the party threads (the Redis mailbox of
// InterimValueCachingService); Castor is a pool of pre-dealt, MAC'd tuple
// streams.  Call for call the same flow as amphora_amd/loopback.py:
//
//   createSecret  DefaultAmphoraClient.java:150-170
//     -> GET /input-masks   InputMaskCachingService.getInputMasksAsOutputDeliveryObject :77-99
//                           (OutputDeliveryService: K_ODO_PRE, open JSON, K_ODO_POST)
//     -> client: verify the mask ODOs + mask the secret (K_MASK)
//     -> POST /masked-inputs  StorageService.createSecret :95-117 -> convertToSecretShare (K_CONV)
//   getSecret     DefaultAmphoraClient.java:206-217
//     -> GET /secret-shares/{id}  OutputDeliveryService.computeOutputDeliveryObject(SecretShare)
//     -> client: recombine + verify (K_RV)
//
// Every word of share arithmetic runs on the GPU; the host code is what a
// JNI-bound Java host would run around it.  Usage:
//   c1_native [words=1024] [reps=20] [shared|own] [parties=2] [pool|fresh]   -> one JSON line
// ("shared": both parties on one context, called from both threads at once;
//  "fresh": a new thread per party per fan-out instead of persistent workers)
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <thread>

#include "amphora.hpp"

using namespace amphora;

namespace {

// Test field of the reference's tests
const u128 P = fromDecimal("198766463529478683931867765928436695041", ~(u128)0);
const u128 R = fromDecimal("141515903391459779531506841503331516415", ~(u128)0);
const u128 RI = fromDecimal("133854242216446749056083838363708373830", ~(u128)0);

// Host Montgomery arithmetic for the dealer (test infrastructure): two
// 64-bit limbs, R = 2^128.  Uniform values are dealt directly in Montgomery
// form ([x] is uniform iff x is), [x][y] -> [xy] by one product.
struct HostMont {
  u128 p;
  uint64_t n0;  // -p^-1 mod 2^64
  explicit HostMont(u128 prime) : p(prime) {
    uint64_t inv = 1, p0 = (uint64_t)prime;
    for (int i = 0; i < 6; ++i) inv *= 2 - p0 * inv;
    n0 = (uint64_t)0 - inv;
  }
  u128 mul(u128 a, u128 b) const {
    const uint64_t b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64), p0 = (uint64_t)p, p1 = (uint64_t)(p >> 64);
    uint64_t t0 = 0, t1 = 0, t2 = 0;
    for (int i = 0; i < 2; ++i) {
      const uint64_t ai = i ? (uint64_t)(a >> 64) : (uint64_t)a;
      u128 c = (u128)ai * b0 + t0;
      t0 = (uint64_t)c;
      c = (u128)ai * b1 + t1 + (c >> 64);
      t1 = (uint64_t)c;
      c = (u128)t2 + (c >> 64);
      t2 = (uint64_t)c;
      const uint64_t t3 = (uint64_t)(c >> 64);
      const uint64_t m = t0 * n0;
      c = (u128)m * p0 + t0;
      c = (u128)m * p1 + t1 + (c >> 64);
      t0 = (uint64_t)c;
      c = (u128)t2 + (c >> 64);
      t1 = (uint64_t)c;
      t2 = t3 + (uint64_t)(c >> 64);
    }
    u128 r = ((u128)t1 << 64) | t0;
    if (t2 || r >= p) r -= p;
    return r;
  }
  u128 sub(u128 a, u128 b) const { return a >= b ? a - b : a + (p - b); }
};

std::string randomUuid(std::mt19937_64& rng) {
  static const char* hex = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < 16; ++i) {
    const unsigned b = (unsigned)(rng() & 0xFF);
    s += hex[b >> 4];
    s += hex[b & 15];
    if (i == 3 || i == 5 || i == 7 || i == 9) s += '-';
  }
  return s;
}

// Castor stand-in: one stream per party of authenticated shares, each
// (requestId, tupleType) dealt once so every party gets its share of the same
// tuples.  Streams are dealt ahead into a pool (deal()) so the timed calls
// only hand them out.
class Dealer {
 public:
  Dealer(int n, const std::vector<u128>& macKeys, uint64_t seed) : n_(n), mont_(P), rng_(seed) {
    u128 a = 0;
    for (u128 k : macKeys) a = addMod(a, k % P, P);
    // [alpha] = alpha * R mod p, by a host double-and-add (once)
    alphaM_ = 0;
    for (int bit = 127; bit >= 0; --bit) {
      alphaM_ = addMod(alphaM_, alphaM_, P);
      if ((R >> bit) & 1) alphaM_ = addMod(alphaM_, a, P);
    }
  }
  void deal(const std::string& type, size_t count, int sets) {
    for (int s = 0; s < sets; ++s) pool_[{type, count}].push_back(make(type, count));
  }
  Bytes operator()(int player, const std::string& id, const std::string& type, size_t count) {
    std::lock_guard<std::mutex> g(mu_);
    auto key = std::make_pair(id, type);
    auto it = dealt_.find(key);
    if (it == dealt_.end()) {
      auto& pl = pool_[{type, count}];
      std::vector<Bytes> st;
      if (pl.empty()) {
        st = make(type, count);
      } else {
        st = std::move(pl.back());
        pl.pop_back();
      }
      it = dealt_.emplace(key, std::make_pair(count, std::move(st))).first;
    }
    if (it->second.first != count) throw std::runtime_error("tuple count mismatch");
    return it->second.second[player];
  }

 private:
  u128 rnd() { return (((u128)rng_() << 64) | rng_()) % P; }
  // value and MAC shares of [x] appended to every party's stream
  void auth(std::vector<Bytes>& st, u128 x) {
    const u128 mac = mont_.mul(alphaM_, x);
    u128 restV = x, restM = mac;
    for (int j = 0; j < n_; ++j) {
      u128 v = restV, m = restM;
      if (j + 1 < n_) {
        v = rnd();
        m = rnd();
        restV = mont_.sub(restV, v);
        restM = mont_.sub(restM, m);
      }
      uint8_t b[32];
      storeLe(v, b);
      storeLe(m, b + 16);
      st[j].insert(st[j].end(), b, b + 32);
    }
  }
  std::vector<Bytes> make(const std::string& type, size_t count) {
    std::vector<Bytes> st(n_);
    for (auto& s : st) s.reserve(count * (type == "INPUT_MASK_GFP" ? 32 : 96));
    for (size_t i = 0; i < count; ++i) {
      if (type == "INPUT_MASK_GFP") {
        auth(st, rnd());
      } else {
        const u128 a = rnd(), b = rnd();
        auth(st, a);
        auth(st, b);
        auth(st, mont_.mul(a, b));
      }
    }
    return st;
  }
  int n_;
  HostMont mont_;
  std::mt19937_64 rng_;
  u128 alphaM_;
  std::mutex mu_;
  std::map<std::pair<std::string, size_t>, std::vector<std::vector<Bytes>>> pool_;
  std::map<std::pair<std::string, std::string>, std::pair<size_t, std::vector<Bytes>>> dealt_;
};

// The inter-VCP open: each party posts its MultiplicationExchangeObject body
// and receives every partner's (OutputDeliveryService.java:201-272).
class Hub {
 public:
  explicit Hub(int n) : n_(n) {}
  std::vector<std::string> exchange(const std::string& body) {
    if (std::getenv("C1_DEBUG"))
      std::fprintf(stderr, "body %zu bytes: %.90s ... %.40s\n", body.size(), body.c_str(),
                   body.size() > 40 ? body.c_str() + body.size() - 40 : body.c_str());
    const std::string op = field(body, "\"operationId\":\"", '"');
    const int pid = std::stoi(field(body, "\"playerId\":", ','));
    std::unique_lock<std::mutex> lk(mu_);
    auto& b = box_[op];
    b.bodies[pid] = body;
    cv_.notify_all();
    if (!cv_.wait_for(lk, std::chrono::seconds(30), [&] { return (int)box_[op].bodies.size() == n_; }))
      throw std::runtime_error("partner diffs for operation " + op + " not received");
    std::vector<std::string> out;
    for (auto& kv : box_[op].bodies)
      if (kv.first != pid) out.push_back(kv.second);
    if (++box_[op].taken == n_) box_.erase(op);
    return out;
  }

 private:
  static std::string field(const std::string& s, const std::string& key, char end) {
    const size_t a = s.find(key);
    if (a == std::string::npos) throw std::runtime_error("exchange body without " + key);
    const size_t b = s.find(end, a + key.size());
    return s.substr(a + key.size(), b - a - key.size());
  }
  struct Entry {
    std::map<int, std::string> bodies;
    int taken = 0;
  };
  int n_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, Entry> box_;
};

// One amphora-service (VCP): its MAC key share, Castor client, input-mask
// cache and secret store, all in memory.
struct Party {
  Party(int id, u128 macKey, const Context& ctx, Dealer& dealer, Hub& hub)
      : id(id), macKey(macKey), ctx(ctx),
        odo(ctx, id, [this, &dealer](const std::string& rid, const std::string& t, size_t c) {
              return dealer(this->id, rid, t, c);
            },
            [&hub](const std::string& body) { return hub.exchange(body); }),
        ssu(ctx) {}
  // GET /input-masks?requestId&count
  OutputDeliveryObject getInputMasks(Dealer& dealer, const std::string& secretId, size_t count) {
    Bytes masks = dealer(id, secretId, "INPUT_MASK_GFP", count);
    OutputDeliveryObject o =
        odo.computeOutputDeliveryObject(masks, 32, nameUUIDFromBytes(secretId + "_odo-computation"));
    std::lock_guard<std::mutex> g(mu);
    maskCache[secretId] = std::move(masks);
    return o;
  }
  // POST /masked-inputs
  void uploadMaskedInput(const std::string& secretId, const std::vector<Bytes>& masked) {
    Bytes masks;
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = maskCache.find(secretId);
      if (it == maskCache.end())
        throw AmphoraServiceException("No input masks found for request ID " + secretId);
      masks = std::move(it->second);
      maskCache.erase(it);
    }
    Bytes share = ssu.convertToSecretShare(masked, toDecimal(macKey), masks, id != 0);
    std::lock_guard<std::mutex> g(mu);
    secrets[secretId] = std::move(share);
  }
  // GET /secret-shares/{id}?requestId
  OutputDeliveryObject getSecretShare(const std::string& secretId, const std::string& requestId) {
    Bytes share;
    {
      std::lock_guard<std::mutex> g(mu);
      share = secrets.at(secretId);
    }
    return odo.computeOutputDeliveryObject(share, 32, requestId);
  }

  int id;
  u128 macKey;
  const Context& ctx;
  service::OutputDeliveryService odo;
  service::SecretShareUtil ssu;
  std::mutex mu;
  std::map<std::string, Bytes> maskCache, secrets;
};

// One call per party on its own thread (AmphoraCommunicationClient's parallel
// fan-out); the first failure is rethrown.  The reference fans out with
// parallelStream, i.e. on the ForkJoin common pool, whose threads persist: so
// each party has ONE persistent worker thread here.  (A fresh std::thread per
// call -- `fresh` on the command line -- pays the HIP runtime's per-thread
// setup on its first call: ~250 us per fan-out, most of a 1 k-word upload;
// rocprofv3 of round 3: hipSetDevice 76 us on average over 664 calls.)
class Worker {
 public:
  Worker() : th_([this] { loop(); }) {}
  ~Worker() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  std::future<void> submit(std::function<void()> f) {
    auto task = std::make_shared<std::packaged_task<void()>>(std::move(f));
    std::future<void> fut = task->get_future();
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return fut;
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  std::thread th_;
};

bool g_fresh_threads = false;
std::vector<std::unique_ptr<Worker>> g_workers;

template <class F>
auto fanOut(std::vector<std::unique_ptr<Party>>& parties, F f) {
  using T = decltype(f(*parties[0]));
  std::vector<T> out(parties.size());
  std::vector<std::exception_ptr> err(parties.size());
  auto job = [&](size_t j) {
    try {
      out[j] = f(*parties[j]);
    } catch (...) {
      err[j] = std::current_exception();
    }
  };
  if (g_fresh_threads) {
    std::vector<std::thread> th;
    for (size_t j = 0; j < parties.size(); ++j) th.emplace_back(job, j);
    for (auto& t : th) t.join();
  } else {
    while (g_workers.size() < parties.size()) g_workers.emplace_back(new Worker());
    std::vector<std::future<void>> done;
    for (size_t j = 0; j < parties.size(); ++j) done.push_back(g_workers[j]->submit([&job, j] { job(j); }));
    for (auto& d : done) d.get();
  }
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
  return out;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void printCauses(const std::exception& e) {
  try {
    std::rethrow_if_nested(e);
  } catch (const std::exception& c) {
    std::fprintf(stderr, "  caused by: %s\n", c.what());
    printCauses(c);
  }
}

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

}  // namespace

int main(int argc, char** argv) {
  const size_t W = argc > 1 ? std::stoul(argv[1]) : 1024;
  const int reps = argc > 2 ? std::stoi(argv[2]) : 20;
  const bool shared = argc > 3 && std::string(argv[3]) == "shared";
  const int n = argc > 4 ? std::stoi(argv[4]) : 2;  // parties
  g_fresh_threads = argc > 5 && std::string(argv[5]) == "fresh";
  const int warm = 3;
  try {
    std::mt19937_64 rng(1);
    std::vector<u128> macKeys;
    for (int j = 0; j < n; ++j) macKeys.push_back((((u128)rng() << 64) | rng()) % P);
    Dealer dealer(n, macKeys, 7);
    Hub hub(n);
    // one context per party (separate services), or "shared": both parties'
    // threads call into one context at the same time (one service's request
    // threads sharing its SecretShareUtil bean)
    std::vector<std::unique_ptr<Context>> ctxs;
    for (int j = 0; j < (shared ? 1 : n); ++j) ctxs.emplace_back(new Context(P, R, RI));
    std::vector<std::unique_ptr<Party>> parties;
    for (int j = 0; j < n; ++j) parties.emplace_back(new Party(j, macKeys[j], *ctxs[shared ? 0 : j], dealer, hub));
    auto util = client::SecretShareUtil::of(P, R, RI);
    // the dealer's Montgomery encoding against the library's toGfp
    {
      HostMont hm(P);
      u128 r2 = 0;  // R^2 mod p = [R]
      for (int bit = 127; bit >= 0; --bit) {
        r2 = addMod(r2, r2, P);
        if ((R >> bit) & 1) r2 = addMod(r2, R, P);
      }
      const std::vector<u128> xs = {0, 1, 90, P - 1, R};
      Bytes g = util.context().toGfp(xs);
      for (size_t i = 0; i < xs.size(); ++i)
        if (loadLe(g.data() + 16 * i) != hm.mul(xs[i], r2)) throw std::runtime_error("dealer encoding differs from toGfp");
    }
    const int total = warm + reps;
    // per upload: W masks (the secret's) + 2W masks and 2W triples (the mask
    // ODO); per download: 2W masks + 2W triples
    dealer.deal("INPUT_MASK_GFP", W, total);
    dealer.deal("INPUT_MASK_GFP", 2 * W, 2 * total);
    dealer.deal("MULTIPLICATION_TRIPLE_GFP", 2 * W, 2 * total);
    std::vector<double> up, down;
    bool exact = true;
    for (int it = 0; it < total; ++it) {
      std::vector<u128> secret(W);
      for (auto& x : secret) x = (((u128)rng() << 64) | rng()) % P;
      const std::string secretId = randomUuid(rng), requestId = randomUuid(rng);
      // createSecret
      auto t0 = std::chrono::steady_clock::now();
      auto maskOdos = fanOut(parties, [&](Party& p) { return std::make_shared<OutputDeliveryObject>(
                                                          p.getInputMasks(dealer, secretId, W)); });
      std::vector<OutputDeliveryObject> mo;
      for (auto& o : maskOdos) mo.push_back(*o);
      const std::vector<Bytes> masked = client::maskSecret(util, secret, mo);
      fanOut(parties, [&](Party& p) { p.uploadMaskedInput(secretId, masked); return 0; });
      const double tu = ms_since(t0);
      // getSecret
      t0 = std::chrono::steady_clock::now();
      auto odos = fanOut(parties, [&](Party& p) { return std::make_shared<OutputDeliveryObject>(
                                                      p.getSecretShare(secretId, requestId)); });
      std::vector<OutputDeliveryObject> so;
      for (auto& o : odos) so.push_back(*o);
      const std::vector<u128> back = client::verifyOutputDeliveryObjects(util, so);
      const double td = ms_since(t0);
      exact = exact && back == secret;
      if (it >= warm) {
        up.push_back(tu);
        down.push_back(td);
      }
    }
    std::printf("{\"tool\": \"c1_native\", \"words\": %zu, \"parties\": %d, \"contexts\": %d, \"reps\": %d, "
                "\"upload_ms_median\": %.3f, \"upload_ms_min\": %.3f, \"download_ms_median\": %.3f, "
                "\"download_ms_min\": %.3f, \"bit_exact_round_trip\": %s, \"fan_out\": \"%s\", \"host\": \"C++ mirror "
                "(include/amphora.hpp), each party on its own thread, JSON open between parties\"}\n",
                W, n, shared ? 1 : n, reps, median(up), *std::min_element(up.begin(), up.end()), median(down),
                *std::min_element(down.begin(), down.end()), exact ? "true" : "false",
                g_fresh_threads ? "a new thread per party per call" : "one persistent worker thread per party");
    return exact ? 0 : 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "c1_native: %s\n", e.what());
    printCauses(e);
    return 2;
  }
}
