// Host-side entropy coder of the bitstream path.
//
// The reference codes its latents with compressai's C++ range-ANS coder
// (models/AutoEncoderRGB_Journal.py:5 imports compressai.ans.BufferedRansEncoder /
// RansDecoder; used at :334,:367-368,:387-388,:401, and by EntropyBottleneck.compress /
// decompress at :319-320,:374) and builds its CDF tables with
// compressai._CXX.pmf_to_quantized_cdf (GaussianConditional / EntropyBottleneck.update,
// called at :309-310,:381).  compressai is not vendored and not installed; this file
// restates its published algorithm (compressai/cpp_exts/rans/rans_interface.cpp over
// ryg_rans' rans64.h, compressai/cpp_exts/ops/ops.cpp) so the byte streams are the same:
//   * 64-bit rANS state, 32-bit renormalisation words, L = 2^31, 16-bit CDF precision;
//   * symbols outside a table's range go through the escape symbol (max_value) followed by
//     4-bit "bypass" digits: the digit count (in runs of 15) then raw_val's nibbles;
//   * the encoder buffers (start, freq, bypass) records and emits them in reverse at flush;
//     the stream is the 32-bit words from the final write pointer to the end, little endian.
// rANS is a single sequential state machine per stream, so this is CPU code: the GPU side
// of the path (symbols, CDF indexes, dequantisation) is csrc/entropy.hip's rgbac_*_code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "common.h"

namespace {

constexpr int kPrecision = 16;                                  // CDF precision (bits)
constexpr int kBypassPrecision = 4;                             // bypass digit width
constexpr uint32_t kMaxBypassVal = (1u << kBypassPrecision) - 1;  // 15
constexpr uint64_t kRansL = 1ull << 31;                         // lower bound of the state

struct RansSym {
  uint16_t start;
  uint16_t range;
  bool bypass;
};

struct Encoder {
  std::vector<RansSym> syms;
};

// Validates one (cdfs, sizes, offsets) table set; returns an error string or nullptr.
const char* check_tables(const int32_t* cdfs, int stride, const int32_t* sizes, int ncdf) {
  if (!cdfs || !sizes || ncdf <= 0 || stride < 3) return "bad CDF table arguments";
  for (int i = 0; i < ncdf; ++i)
    if (sizes[i] < 3 || sizes[i] > stride) return "CDF length out of range";
  return nullptr;
}

// rans_interface.cpp, BufferedRansEncoder::encode_with_indexes
int encode_into(Encoder& enc, const int32_t* symbols, const int32_t* indexes, int64_t n,
                const int32_t* cdfs, int stride, const int32_t* sizes, const int32_t* offsets,
                int ncdf) {
  for (int64_t i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    if (ci < 0 || ci >= ncdf) {
      rgbac::set_error("rgbac_rans_encoder_put: CDF index out of range");
      return RGBAC_E_ARG;
    }
    const int32_t* cdf = cdfs + (int64_t)ci * stride;
    const int32_t max_value = sizes[ci] - 2;
    int32_t value = symbols[i] - offsets[ci];
    uint32_t raw_val = 0;
    if (value < 0) {
      raw_val = (uint32_t)(-2 * (int64_t)value - 1);
      value = max_value;
    } else if (value >= max_value) {
      raw_val = (uint32_t)(2 * (int64_t)(value - max_value));
      value = max_value;
    }
    enc.syms.push_back({(uint16_t)cdf[value], (uint16_t)(cdf[value + 1] - cdf[value]), false});
    if (value == max_value) {
      int32_t n_bypass = 0;
      while (n_bypass < 8 && (raw_val >> (n_bypass * kBypassPrecision)) != 0) ++n_bypass;
      int32_t val = n_bypass;
      while (val >= (int32_t)kMaxBypassVal) {
        enc.syms.push_back({(uint16_t)kMaxBypassVal, (uint16_t)(kMaxBypassVal + 1), true});
        val -= kMaxBypassVal;
      }
      enc.syms.push_back({(uint16_t)val, (uint16_t)(val + 1), true});
      for (int32_t j = 0; j < n_bypass; ++j) {
        const uint32_t v = (raw_val >> (j * kBypassPrecision)) & kMaxBypassVal;
        enc.syms.push_back({(uint16_t)v, (uint16_t)(v + 1), true});
      }
    }
  }
  return 0;
}

// rans64.h Rans64EncPut
inline void enc_put(uint64_t& x, uint32_t*& ptr, uint32_t start, uint32_t freq) {
  const uint64_t x_max = ((kRansL >> kPrecision) << 32) * freq;
  if (x >= x_max) {
    *--ptr = (uint32_t)x;
    x >>= 32;
  }
  x = ((x / freq) << kPrecision) + (x % freq) + start;
}

// rans_interface.cpp Rans64EncPutBits
inline void enc_put_bits(uint64_t& x, uint32_t*& ptr, uint32_t val, uint32_t nbits) {
  const uint32_t freq = 1u << (16 - nbits);
  const uint64_t x_max = ((kRansL >> 16) << 32) * freq;
  if (x >= x_max) {
    *--ptr = (uint32_t)x;
    x >>= 32;
  }
  x = (x << nbits) | val;
}

}  // namespace

extern "C" int rgbac_pmf_to_quantized_cdf(const float* pmf, int n, int precision,
                                          uint32_t* cdf) {
  // compressai/cpp_exts/ops/ops.cpp pmf_to_quantized_cdf: round p * 2^precision, rescale to
  // the exact total, then give every zero-frequency symbol one count stolen from the
  // smallest frequency > 1.
  RGBAC_REQUIRE(pmf && cdf && n > 0, "null pointer / empty pmf");
  RGBAC_REQUIRE(precision > 0 && precision <= 16, "precision");
  for (int i = 0; i < n; ++i)
    RGBAC_REQUIRE(pmf[i] >= 0.0f && std::isfinite(pmf[i]), "invalid `pmf`, non-finite or negative");
  const uint32_t one = 1u << precision;
  std::vector<uint32_t> c(n + 1);
  c[0] = 0;
  for (int i = 0; i < n; ++i) c[i + 1] = (uint32_t)std::round(pmf[i] * (float)one);
  uint32_t total = 0;
  for (uint32_t v : c) total += v;
  RGBAC_REQUIRE(total != 0, "invalid `pmf`: at least one element must have a non-zero probability");
  for (auto& v : c) v = (uint32_t)(((uint64_t)one * v) / total);
  for (int i = 1; i <= n; ++i) c[i] += c[i - 1];
  c[n] = one;
  for (int i = 0; i < n; ++i) {
    if (c[i] == c[i + 1]) {
      uint32_t best_freq = ~0u;
      int best_steal = -1;
      for (int j = 0; j < n; ++j) {
        const uint32_t f = c[j + 1] - c[j];
        if (f > 1 && f < best_freq) {
          best_freq = f;
          best_steal = j;
        }
      }
      RGBAC_REQUIRE(best_steal != -1, "no frequency left to steal");
      if (best_steal < i) {
        for (int j = best_steal + 1; j <= i; ++j) c[j]--;
      } else {
        for (int j = i + 1; j <= best_steal; ++j) c[j]++;
      }
    }
  }
  std::memcpy(cdf, c.data(), sizeof(uint32_t) * (n + 1));
  return 0;
}

extern "C" int rgbac_rans_encoder_create(void** handle) {
  RGBAC_REQUIRE(handle, "null pointer");
  *handle = new (std::nothrow) Encoder();
  RGBAC_REQUIRE(*handle, "out of host memory");
  return 0;
}

extern "C" int rgbac_rans_encoder_destroy(void* handle) {
  delete static_cast<Encoder*>(handle);
  return 0;
}

extern "C" int rgbac_rans_encoder_put(void* handle, const int32_t* symbols,
                                      const int32_t* indexes, int64_t n, const int32_t* cdfs,
                                      int cdf_stride, const int32_t* cdf_sizes,
                                      const int32_t* offsets, int ncdf) {
  RGBAC_REQUIRE(handle && offsets && (n == 0 || (symbols && indexes)), "null pointer");
  RGBAC_REQUIRE(n >= 0, "negative symbol count");
  const char* bad = check_tables(cdfs, cdf_stride, cdf_sizes, ncdf);
  RGBAC_REQUIRE(!bad, bad ? bad : "");
  Encoder& enc = *static_cast<Encoder*>(handle);
  const size_t mark = enc.syms.size();
  const int rc = encode_into(enc, symbols, indexes, n, cdfs, cdf_stride, cdf_sizes, offsets, ncdf);
  if (rc != 0) enc.syms.resize(mark);  // a failed put leaves the encoder unchanged
  return rc;
}

extern "C" int64_t rgbac_rans_encoder_bound(void* handle) {
  // every buffered record emits at most one 32-bit word, plus the 64-bit final state
  if (!handle) return -1;
  return ((int64_t)static_cast<Encoder*>(handle)->syms.size() + 2) * 4;
}

extern "C" int rgbac_rans_encoder_flush(void* handle, uint8_t* out, int64_t capacity,
                                        int64_t* nbytes) {
  // rans_interface.cpp BufferedRansEncoder::flush: encode the records last-to-first, then
  // Rans64EncFlush; the encoder is empty afterwards.
  RGBAC_REQUIRE(handle && out && nbytes, "null pointer");
  Encoder& enc = *static_cast<Encoder*>(handle);
  const int64_t words = (int64_t)enc.syms.size() + 2;
  RGBAC_REQUIRE(capacity >= words * 4, "output buffer smaller than rgbac_rans_encoder_bound");
  std::vector<uint32_t> buf((size_t)words);
  uint32_t* end = buf.data() + buf.size();
  uint32_t* ptr = end;
  uint64_t x = kRansL;
  for (auto it = enc.syms.rbegin(); it != enc.syms.rend(); ++it) {
    if (!it->bypass)
      enc_put(x, ptr, it->start, it->range);
    else
      enc_put_bits(x, ptr, it->start, kBypassPrecision);
  }
  ptr -= 2;
  ptr[0] = (uint32_t)x;
  ptr[1] = (uint32_t)(x >> 32);
  const int64_t nb = (int64_t)(end - ptr) * 4;
  std::memcpy(out, ptr, (size_t)nb);  // little-endian words, as compressai's std::string
  *nbytes = nb;
  enc.syms.clear();
  return 0;
}

namespace {

inline int dec_word(rgbac_rans_decoder_t* d, uint32_t* w) {
  if (d->pos + 4 > d->size) return -1;
  std::memcpy(w, d->data + d->pos, 4);
  d->pos += 4;
  return 0;
}

// rans_interface.cpp Rans64DecGetBits
inline int dec_get_bits(rgbac_rans_decoder_t* d, uint32_t nbits, uint32_t* val) {
  uint64_t x = d->state;
  *val = (uint32_t)(x & ((1u << nbits) - 1));
  x >>= nbits;
  if (x < kRansL) {
    uint32_t w;
    if (dec_word(d, &w)) return -1;
    x = (x << 32) | w;
  }
  d->state = x;
  return 0;
}

}  // namespace

extern "C" int rgbac_rans_decoder_init(rgbac_rans_decoder_t* d, const uint8_t* data,
                                       int64_t nbytes) {
  // RansDecoder::set_stream + Rans64DecInit
  RGBAC_REQUIRE(d && data, "null pointer");
  RGBAC_REQUIRE(nbytes >= 8 && nbytes % 4 == 0, "stream length must be a multiple of 4, >= 8");
  d->data = data;
  d->size = nbytes;
  d->pos = 0;
  uint32_t lo, hi;
  dec_word(d, &lo);
  dec_word(d, &hi);
  d->state = (uint64_t)lo | ((uint64_t)hi << 32);
  return 0;
}

extern "C" int rgbac_rans_decode(rgbac_rans_decoder_t* d, const int32_t* indexes, int64_t n,
                                 const int32_t* cdfs, int cdf_stride, const int32_t* cdf_sizes,
                                 const int32_t* offsets, int ncdf, int32_t* out) {
  // RansDecoder::decode_stream: locate cum_freq in the index's CDF (first entry > cum_freq;
  // the tables are increasing, so a binary search finds the same slot as compressai's
  // linear scan), advance, and undo the escape/bypass coding.
  RGBAC_REQUIRE(d && d->data && offsets && (n == 0 || (indexes && out)), "null pointer");
  RGBAC_REQUIRE(n >= 0, "negative symbol count");
  const char* bad = check_tables(cdfs, cdf_stride, cdf_sizes, ncdf);
  RGBAC_REQUIRE(!bad, bad ? bad : "");
  const uint32_t mask = (1u << kPrecision) - 1;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    RGBAC_REQUIRE(ci >= 0 && ci < ncdf, "CDF index out of range");
    const int32_t* cdf = cdfs + (int64_t)ci * cdf_stride;
    const int32_t size = cdf_sizes[ci];
    const int32_t max_value = size - 2;
    const uint32_t cum = (uint32_t)(d->state & mask);
    const int32_t* it = std::upper_bound(cdf, cdf + size, (int32_t)cum);
    RGBAC_REQUIRE(it != cdf && it != cdf + size, "corrupt stream or CDF table");
    const int32_t s = (int32_t)(it - cdf) - 1;
    const uint32_t start = (uint32_t)cdf[s], freq = (uint32_t)(cdf[s + 1] - cdf[s]);
    uint64_t x = d->state;
    x = freq * (x >> kPrecision) + (x & mask) - start;
    if (x < kRansL) {
      uint32_t w;
      RGBAC_REQUIRE(dec_word(d, &w) == 0, "read past the end of the stream");
      x = (x << 32) | w;
    }
    d->state = x;
    int32_t value = s;
    if (value == max_value) {
      uint32_t val;
      RGBAC_REQUIRE(dec_get_bits(d, kBypassPrecision, &val) == 0, "read past the end of the stream");
      int32_t n_bypass = (int32_t)val;
      while (val == kMaxBypassVal) {
        RGBAC_REQUIRE(dec_get_bits(d, kBypassPrecision, &val) == 0,
                      "read past the end of the stream");
        n_bypass += (int32_t)val;
      }
      RGBAC_REQUIRE(n_bypass <= 8, "corrupt bypass length");
      uint32_t raw_val = 0;
      for (int32_t j = 0; j < n_bypass; ++j) {
        RGBAC_REQUIRE(dec_get_bits(d, kBypassPrecision, &val) == 0,
                      "read past the end of the stream");
        raw_val |= val << (j * kBypassPrecision);
      }
      value = (int32_t)(raw_val >> 1);
      if (raw_val & 1)
        value = -value - 1;
      else
        value += max_value;
    }
    out[i] = value + offsets[ci];
  }
  return 0;
}
