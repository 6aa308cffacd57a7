// Launch interface of the share-arithmetic kernels (internal to libamphora_hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "field.hpp"

namespace amph {

constexpr int kMaxParties = 16;
constexpr int kMaxBlock = 1024;  // kernels accept any block size <= this
// first_fail sentinel: what hipMemsetAsync(.., 0x7F, 8) leaves behind.
constexpr unsigned long long kNoFail = 0x7F7F7F7F7F7F7F7FULL;

// SoA word arrays of one OutputDeliveryObject set: f[field][party], field
// order y (secretShares), r, v, w, u.  Each points at 16-byte words.
struct OdoSet {
  const uint4* f[5][kMaxParties];
};

struct ShareSet {
  const uint4* s[kMaxParties];
};

// The exchange decode's SPAN FORM (launch_exchange_decode_spans): the values
// of 8 KiB span s of the text, in text order, at slots [kXSpanSlots s, ...);
// neg byte per slot = sign (bit 0) | key "b" (bit 1).  base[s] = the index of
// span s's first value (bits 0..39), base[nb] = the total; when base[nb]
// carries bits above 39 or its count is not the pair count x 2, the general
// pass wrote the values in pair order instead (slot = value index).  map[b]
// = the window of values [kXMapValues b, kXMapValues (b + 1)) (one
// k_open_post workgroup's): x = s0, the span holding its first value, y = that
// value's rank in s0, z = o1 | o2 << 16, w = o3 with o_i = base[s0 + i] -
// kXMapValues b (0xFFFF / ~0 past the last span): value kXMapValues b + t
// lies in span s0 + i for o_i <= t < o_(i+1) (o_0 = -y).
constexpr size_t kXSpanBytes = 8192;
constexpr int kXSpanSlots = 528;  // 33 x 256 B per span: not a power-of-two stride (see k_xdec_span)
constexpr size_t kXMapValues = 256;
struct XSpans {
  uint4* mag;
  uint8_t* neg;
  uint64_t* base;  // nb + 1 words
  uint4* map;      // xspan_map_words(npairs) windows
  size_t nb;       // xspan_spans(len)
};

struct SignedSet {  // per party: diff magnitudes (2 words per pair) + sign words
  const uint4* mag[kMaxParties];
  const uint32_t* neg[kMaxParties];  // 4 sign bytes per source word (see K_ODO_PRE)
  // span form (k_open_post only): base / map / nb of the party's XSpans, null
  // for pair-ordered diffs (amph_odo_pre's layout)
  const uint64_t* sbase[kMaxParties];
  const uint4* smap[kMaxParties];
  size_t snb[kMaxParties];
};

struct TextSet {  // base64 text of each ODO field: t[field][party], 16-byte aligned
  const char* t[5][kMaxParties];
};

struct LaunchCfg {
  hipStream_t stream;
  int grid_cap;  // 0 = full grid (one word per thread); > 0 caps it (grid-stride beyond)
  int block;     // threads per workgroup, multiple of 64, <= kMaxBlock
  hipEvent_t ev_start = nullptr;  // optional: stamped by the kernel dispatch itself
  hipEvent_t ev_stop = nullptr;
};

// K_RV: recombine 5 fields over n parties, verify w == y r, u == v r,
// write canonical y (LE16) and atomic-min the first failing index.
hipError_t launch_recombine_verify(const OdoSet& odo, int n, size_t words, uint4* out_y,
                                   unsigned long long* first_fail, const Fp& f, const LaunchCfg& c);

// K_MASK: K_RV over Input Mask ODOs fused with maskInput:
// out[i] = [s_i] - [m_i] for i < n_secrets (s_i any 128-bit LE integer).
hipError_t launch_mask_input(const OdoSet& odo, int n, size_t words, const uint4* secrets,
                             size_t n_secrets, uint4* out_masked, unsigned long long* first_fail,
                             const Fp& f, const LaunchCfg& c);

// recombineObject for one field: canonical sum_j fromGfp(share_j).
hipError_t launch_recombine(const ShareSet& sh, int n, size_t words, uint4* out, const Fp& f,
                            const LaunchCfg& c);

// verifySecrets on canonical (LE16) integers: y r == w and v r == u (mod p).
// min-combine a one-word call's verdict (index 0 or kNoFail) as word `base`
hipError_t launch_ff_merge(unsigned long long* ff, const unsigned long long* tail, size_t base,
                           hipStream_t s);

hipError_t launch_verify(const uint4* y, const uint4* r, const uint4* u, const uint4* v,
                         const uint4* w, size_t words, unsigned long long* first_fail,
                         const Fp& f, const LaunchCfg& c);

// K_CONV: masked (16 B) + input-mask tuple (value||mac, 32 B) -> share (value||mac).
hipError_t launch_convert_share(const uint4* masked, const uint4* tuples, size_t words,
                                W4 alpha_mont, int use_zero_input, uint4* out, const Fp& f,
                                const LaunchCfg& c);

// K_ODO_PRE: raw y/r/v copies (each optional) + signed Beaver diffs; with
// lens, also the exchange text length of every kXLenPairs FactorPairs
// (launch_exchange_encode_lens' input).
constexpr size_t kXLenPairs = 128;
hipError_t launch_odo_pre(const uint4* share_data, int share_stride_words, const uint4* masks,
                          const uint4* triples, size_t words, uint4* out_y, uint4* out_r,
                          uint4* out_v, uint4* out_mag, uint32_t* out_neg, const Fp& f,
                          const LaunchCfg& c, uint64_t* lens = nullptr);

// recombineDiffs: sum over parties of signed diffs mod p -> canonical opened values.
hipError_t launch_open_diffs(const SignedSet& d, int n, size_t pairs, uint4* out_opened,
                             const Fp& f, const LaunchCfg& c);

// K_ODO_POST: Beaver product shares from opened (D, E) + triples -> w, u wire words.
hipError_t launch_odo_post(const uint4* opened, const uint4* triples, size_t words,
                           int is_player0, uint4* out_w, uint4* out_u, const Fp& f,
                           const LaunchCfg& c);

// recombineDiffs + K_ODO_POST in one launch: every party's signed diffs
// (SignedSet) + triples -> w, u wire words; the opened D, E stay in registers.
hipError_t launch_open_post(const SignedSet& d, int n, const uint4* triples, size_t words,
                            int is_player0, uint4* out_w, uint4* out_u, const Fp& f,
                            const LaunchCfg& c, bool stage_mag = false);

// toGfp / fromGfp over word arrays; maskInput with canonical masks.
hipError_t launch_to_gfp(const uint4* in, size_t words, uint4* out, const Fp& f, const LaunchCfg& c);
hipError_t launch_from_gfp(const uint4* in, size_t words, uint4* out, const Fp& f, const LaunchCfg& c);
hipError_t launch_mask_words(const uint4* secrets, const uint4* masks, size_t words, uint4* out,
                             const Fp& f, const LaunchCfg& c);

// base64 wire codec (codec.hip): standard alphabet, '=' padding, no line breaks.
hipError_t launch_b64_encode(const uint8_t* in, size_t nbytes, char* out, const LaunchCfg& c);
// n <= 5 streams of nbytes each, one launch
hipError_t launch_b64_encode_multi(const uint8_t* const* in, char* const* out, int n, size_t nbytes,
                                   const LaunchCfg& c);
// text_end: the range ends the text, so '=' may pad its last two chars;
// out_bytes = kB64PadOnDevice (with text_end): the kernel sizes the output
// from the text's last two characters itself, no host read-back
constexpr size_t kB64PadOnDevice = ~(size_t)0;
hipError_t launch_b64_decode(const char* in, size_t nchars, uint8_t* out, size_t out_bytes,
                             unsigned long long* bad, const LaunchCfg& c, bool text_end = true);
hipError_t launch_b64_words(const uint4* in, size_t words, char* out, const LaunchCfg& c);
hipError_t launch_b64_unwords(const char* in, size_t words, uint4* out, unsigned long long* bad,
                              const LaunchCfg& c);

// Beaver open exchange codec (exchange.hip): FactorPair JSON array <-> signed
// diffs (mag 16 B + sign byte per value, 2 values per pair).
size_t xenc_scratch_bytes(size_t npairs);
size_t xenc_max_bytes(size_t npairs);
hipError_t launch_exchange_encode(const uint4* mag, const uint8_t* neg, size_t npairs, char* out,
                                  unsigned long long* out_len, void* scratch, const LaunchCfg& c);
// the same text when K_ODO_PRE has written the lengths of every kXLenPairs
// pairs (lens: ceil(npairs / kXLenPairs) + 1 words, scanned in place)
size_t xenc_lens_scratch_bytes(size_t npairs);
hipError_t launch_exchange_encode_lens(const uint4* mag, const uint8_t* neg, size_t npairs, uint64_t* lens,
                                       char* out, unsigned long long* out_len, void* scratch, const LaunchCfg& c);
size_t xdec_scratch_bytes(size_t len);
hipError_t launch_exchange_decode(const char* text, size_t len, size_t npairs, uint4* mag,
                                  uint8_t* neg, unsigned long long* bad, void* scratch,
                                  const LaunchCfg& c);
// decode into span form (see XSpans): one read of the text, no count pass;
// resets *bad itself (kNoFail) before reporting into it
size_t xspan_spans(size_t len);
size_t xspan_slots(size_t len, size_t npairs);  // >= both the span slots and 2 npairs
size_t xspan_map_words(size_t npairs);
size_t xdec_spans_scratch_bytes(size_t len);
hipError_t launch_exchange_decode_spans(const char* text, size_t len, size_t npairs, const XSpans& out,
                                        unsigned long long* bad, void* scratch, const LaunchCfg& c);

// Synthetic honest n-party ODOs (bench/test input generator, device-side).
struct OutSet {
  uint4* f[5][kMaxParties];
};
hipError_t launch_synth_odos(const OutSet& out, int n, size_t words, uint64_t seed,
                             uint4* out_plain_y, long long fault_index, int noncanon_permille,
                             const Fp& f, const LaunchCfg& c);
hipError_t launch_synth_words(uint4* out, size_t count, uint64_t seed, const Fp& f,
                              const LaunchCfg& c);
// K_RV / K_MASK straight from the wire: the parties' base64 ODO fields
// (nchars each = 4 ceil(16 words / 3), `pad` '=' at the end) decoded in the
// workgroup; bad = min (5 party + field) * nchars + offset of an invalid char.
hipError_t launch_rv_b64(const TextSet& tx, int n, size_t words, size_t nchars, uint32_t pad,
                         uint4* out_y, unsigned long long* first_fail, unsigned long long* bad,
                         const Fp& f, const LaunchCfg& c);
hipError_t launch_mask_b64(const TextSet& tx, int n, size_t words, size_t nchars, uint32_t pad,
                           const uint4* secrets, size_t n_secrets, uint4* out16, char* out24,
                           unsigned long long* first_fail, unsigned long long* bad, const Fp& f,
                           const LaunchCfg& c);

// Small host calls: copy n verdict words from device memory to page-locked
// host memory and reset them to kNoFail (one 64-lane workgroup).
hipError_t launch_take_words(unsigned long long* dev, unsigned long long* host, int n, hipStream_t s);

// Device-mode party session: poison the five base64 fields ("!!!!" as their
// first unit) when any partner verdict word is not kNoFail (one workgroup).
struct PoisonB64 {
  const unsigned long long* bad[16];
  int n_bad;
  char* field[5];
  size_t chars;  // characters per field
};
hipError_t launch_poison_b64(const PoisonB64& a, hipStream_t s);

// Measurement only: K_MASK's memory pattern without the arithmetic.
hipError_t launch_stream_probe(const OdoSet& odo, int n, size_t words, const uint4* secrets,
                               uint4* out, const LaunchCfg& c);

}  // namespace amph
