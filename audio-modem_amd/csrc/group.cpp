// group.cpp — one host process driving several GPUs (the Node host
// decoding one batch on N devices). A group holds one context per device; a batch is cut
// into contiguous frame ranges of about equal sample counts, each range decoded on its own
// device concurrently (host thread per device: H2D of the range's samples, the fast and
// exact kernels, D2H of its results straight into the caller's arrays). Frames are
// independent, so there is no device-to-device exchange on the data path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "amodem_internal.h"

struct amod_group {
  std::vector<amod_ctx *> ctx;
};

namespace {
// contiguous frame ranges of about equal sample counts: member k takes [cut[k], cut[k+1])
std::vector<int32_t> split_frames(const int32_t *lengths, int32_t nframes, int nd) {
  std::vector<int64_t> cum((size_t)nframes + 1, 0);
  for (int32_t i = 0; i < nframes; ++i) cum[(size_t)i + 1] = cum[(size_t)i] + lengths[i];
  std::vector<int32_t> cut((size_t)nd + 1, 0);
  for (int k = 1; k < nd; ++k) {
    const int64_t want = cum.back() * k / nd;
    cut[(size_t)k] = (int32_t)(std::lower_bound(cum.begin(), cum.end(), want) - cum.begin());
    cut[(size_t)k] = std::max(cut[(size_t)k - 1], std::min(cut[(size_t)k], nframes));
  }
  cut[(size_t)nd] = nframes;
  return cut;
}
// the samples a frame range spans, [lo, hi), lo rounded down to a multiple of 4 so every
// frame keeps its offset mod 4 (the fast path's block moments sit on 16-byte boundaries of
// the buffer, so its approximate coarse_idx follows the alignment)
void span_of(const int64_t *offsets, const int32_t *lengths, int32_t a, int32_t b, int64_t &lo, int64_t &hi) {
  lo = INT64_MAX;
  hi = 0;
  for (int32_t i = a; i < b; ++i) { lo = std::min(lo, offsets[i]); hi = std::max(hi, offsets[i] + lengths[i]); }
  lo &= ~int64_t(3);
}
} // namespace

extern "C" int amod_group_open(const int32_t *devices, int32_t ndev, amod_group **out) {
  if (!out || !devices || ndev < 1 || ndev > 64) return amod_ctx_fail(nullptr, "invalid group arguments", AMOD_ERR_ARG);
  auto *g = new amod_group;
  for (int32_t i = 0; i < ndev; ++i) {
    amod_ctx *c = nullptr;
    const int rc = amod_open(devices[i], &c);
    if (rc != AMOD_SUCCESS) {
      for (auto *p : g->ctx) amod_close(p);
      delete g;
      return rc;
    }
    g->ctx.push_back(c);
  }
  *out = g;
  return AMOD_SUCCESS;
}

extern "C" int amod_group_close(amod_group *g) {
  if (!g) return AMOD_SUCCESS;
  for (auto *c : g->ctx) amod_close(c);
  delete g;
  return AMOD_SUCCESS;
}

extern "C" int32_t amod_group_size(const amod_group *g) { return g ? (int32_t)g->ctx.size() : 0; }

extern "C" amod_ctx *amod_group_context(amod_group *g, int32_t i) {
  return (g && i >= 0 && i < (int32_t)g->ctx.size()) ? g->ctx[(size_t)i] : nullptr;
}

extern "C" int amod_group_decode_host(amod_group *g, const amod_cfg *cfg, int32_t mode, const float *samples,
                                      int64_t nsamples, const int64_t *offsets, const int32_t *lengths,
                                      int32_t nframes, amod_result *results, uint8_t *payload, int64_t payload_stride,
                                      uint32_t options, int32_t *frames_per_device) {
  if (!g || g->ctx.empty()) return amod_ctx_fail(nullptr, "null group", AMOD_ERR_ARG);
  if (nframes < 0 || nsamples < 0 || (nframes && (!offsets || !lengths || !results || !payload)))
    return amod_ctx_fail(nullptr, "invalid argument", AMOD_ERR_ARG);
  for (int32_t i = 0; i < nframes; ++i)
    if (offsets[i] < 0 || lengths[i] < 0 || offsets[i] + lengths[i] > nsamples)
      return amod_ctx_fail(nullptr, ("frame " + std::to_string(i) + " lies outside the sample buffer").c_str(),
                           AMOD_ERR_ARG);
  const int nd = (int)g->ctx.size();
  const std::vector<int32_t> cut = split_frames(lengths, nframes, nd);
  std::vector<int> rc((size_t)nd, AMOD_SUCCESS);
  std::vector<std::string> err((size_t)nd);
  std::vector<std::thread> th;
  for (int k = 0; k < nd; ++k) {
    const int32_t a = cut[(size_t)k], b = cut[(size_t)k + 1];
    if (frames_per_device) frames_per_device[k] = b - a;
    if (b <= a) continue;
    th.emplace_back([&, k, a, b] {
      int64_t lo, hi;
      span_of(offsets, lengths, a, b, lo, hi);
      std::vector<int64_t> loc((size_t)(b - a));
      for (int32_t i = a; i < b; ++i) loc[(size_t)(i - a)] = offsets[i] - lo;
      rc[(size_t)k] = amod_decode_host(g->ctx[(size_t)k], cfg, mode, samples + lo, hi - lo, loc.data(), lengths + a,
                                       b - a, results + a, payload + (size_t)a * (size_t)payload_stride,
                                       payload_stride, options);
      if (rc[(size_t)k] != AMOD_SUCCESS) err[(size_t)k] = amod_last_error(g->ctx[(size_t)k]);
    });
  }
  for (auto &t : th) t.join();
  for (int k = 0; k < nd; ++k)
    if (rc[(size_t)k] != AMOD_SUCCESS)
      return amod_ctx_fail(nullptr, ("device " + std::to_string(k) + ": " + err[(size_t)k]).c_str(), rc[(size_t)k]);
  return AMOD_SUCCESS;
}

// ------------------------------------------------------------ device-resident shards
extern "C" int amod_group_decode_device(amod_group *g, const amod_cfg *cfg, int32_t mode, const amod_shard *shards,
                                        uint32_t options) {
  if (!g || g->ctx.empty() || !shards) return amod_ctx_fail(nullptr, "invalid group arguments", AMOD_ERR_ARG);
  for (size_t k = 0; k < g->ctx.size(); ++k) {
    const amod_shard &sh = shards[k];
    if (sh.nframes < 0) return amod_ctx_fail(nullptr, "shard nframes < 0", AMOD_ERR_ARG);
    if (sh.nframes == 0) continue;
    const int rc = amod_decode_device(g->ctx[k], cfg, mode, sh.samples, sh.offsets, sh.lengths, sh.nframes, sh.results,
                                      sh.payload, sh.payload_stride, options, sh.stream);
    if (rc != AMOD_SUCCESS)
      return amod_ctx_fail(nullptr, ("device " + std::to_string(k) + ": " + amod_last_error(g->ctx[k])).c_str(), rc);
  }
  return AMOD_SUCCESS;
}

extern "C" int amod_group_synchronize(amod_group *g) {
  if (!g) return amod_ctx_fail(nullptr, "null group", AMOD_ERR_ARG);
  for (auto *c : g->ctx) {
    const int rc = amod_synchronize(c);
    if (rc != AMOD_SUCCESS) return rc;
  }
  return AMOD_SUCCESS;
}

// one member's resident shard: the range's samples (from lo), frame offsets relative to
// lo, lengths, and the result / payload buffers of the latest decode's stride
struct ResidentShard {
  int device = 0;
  int32_t first = 0, nframes = 0;
  void *samples = nullptr, *offsets = nullptr, *lengths = nullptr, *results = nullptr, *payload = nullptr;
  size_t payload_bytes = 0;
};

struct amod_resident {
  // one decode at a time: every decode of the batch shares its shards' device result and
  // payload buffers (and may reallocate the payload), and the Node addon runs decodes on
  // the libuv pool, so two outstanding decodeBatch(DeviceBatch) calls would race
  std::mutex mu;
  amod_group *g = nullptr;
  int32_t nframes = 0;
  int32_t max_len = 0;
  std::vector<ResidentShard> sh;
};

static void free_shard(ResidentShard &s) {
  (void)hipSetDevice(s.device);
  for (void *p : {s.samples, s.offsets, s.lengths, s.results, s.payload})
    if (p) (void)hipFree(p);
  s = ResidentShard{};
}

extern "C" int amod_resident_free(amod_resident *r) {
  if (!r) return AMOD_SUCCESS;
  for (auto &s : r->sh) free_shard(s);
  delete r;
  return AMOD_SUCCESS;
}

#define G_TRY(expr, r)                                                                     \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      amod_resident_free(r);                                                               \
      return amod_ctx_fail(nullptr, (std::string(#expr) + ": " + hipGetErrorString(e_)).c_str(), AMOD_ERR_HIP); \
    }                                                                                      \
  } while (0)

extern "C" int amod_group_upload(amod_group *g, const amod_cfg *cfg, const float *samples, int64_t nsamples,
                                 const int64_t *offsets, const int32_t *lengths, int32_t nframes, amod_resident **out) {
  if (!g || g->ctx.empty() || !out || !cfg || nframes < 0 || nsamples < 0 ||
      (nframes && (!offsets || !lengths || !samples)))
    return amod_ctx_fail(nullptr, "invalid argument", AMOD_ERR_ARG);
  if (!amod_cfg_valid(cfg)) return amod_ctx_fail(nullptr, "invalid amod_cfg", AMOD_ERR_ARG);
  for (int32_t i = 0; i < nframes; ++i)
    if (offsets[i] < 0 || lengths[i] < 0 || offsets[i] + lengths[i] > nsamples)
      return amod_ctx_fail(nullptr, ("frame " + std::to_string(i) + " lies outside the sample buffer").c_str(),
                           AMOD_ERR_ARG);
  const int nd = (int)g->ctx.size();
  const std::vector<int32_t> cut = split_frames(lengths, nframes, nd);
  auto *r = new amod_resident;
  r->g = g;
  r->nframes = nframes;
  for (int32_t i = 0; i < nframes; ++i) r->max_len = std::max(r->max_len, lengths[i]);
  r->sh.resize((size_t)nd);
  for (int k = 0; k < nd; ++k) {
    ResidentShard &s = r->sh[(size_t)k];
    s.device = amod_ctx_device(g->ctx[(size_t)k]);
    s.first = cut[(size_t)k];
    s.nframes = cut[(size_t)k + 1] - s.first;
    if (s.nframes <= 0) continue;
    int64_t lo, hi;
    span_of(offsets, lengths, s.first, s.first + s.nframes, lo, hi);
    std::vector<int64_t> loc((size_t)s.nframes);
    int32_t ml = 0;
    for (int32_t i = 0; i < s.nframes; ++i) {
      loc[(size_t)i] = offsets[s.first + i] - lo;
      ml = std::max(ml, lengths[s.first + i]);
    }
    G_TRY(hipSetDevice(s.device), r);
    G_TRY(hipMalloc(&s.samples, sizeof(float) * (size_t)(hi - lo + 4)), r);
    G_TRY(hipMalloc(&s.offsets, sizeof(int64_t) * (size_t)s.nframes), r);
    G_TRY(hipMalloc(&s.lengths, sizeof(int32_t) * (size_t)s.nframes), r);
    G_TRY(hipMalloc(&s.results, sizeof(amod_result) * (size_t)s.nframes), r);
    G_TRY(hipMemcpy(s.samples, samples + lo, sizeof(float) * (size_t)(hi - lo), hipMemcpyHostToDevice), r);
    G_TRY(hipMemcpy(s.offsets, loc.data(), sizeof(int64_t) * (size_t)s.nframes, hipMemcpyHostToDevice), r);
    G_TRY(hipMemcpy(s.lengths, lengths + s.first, sizeof(int32_t) * (size_t)s.nframes, hipMemcpyHostToDevice), r);
    // the member's device path sized for this shard (fast-path capacity and workspace)
    const int rc = amod_reserve(g->ctx[(size_t)k], cfg, s.nframes, ml);
    if (rc != AMOD_SUCCESS) {
      amod_resident_free(r);
      return rc;
    }
  }
  *out = r;
  return AMOD_SUCCESS;
}

extern "C" int32_t amod_resident_frames(const amod_resident *r, int32_t *frames_per_device) {
  if (!r) return 0;
  if (frames_per_device)
    for (size_t k = 0; k < r->sh.size(); ++k) frames_per_device[k] = r->sh[k].nframes;
  return r->nframes;
}

extern "C" int amod_resident_decode(amod_resident *r, const amod_cfg *cfg, int32_t mode, uint32_t options,
                                    amod_result *results, uint8_t *payload, int64_t payload_stride) {
  if (!r || !cfg || (r->nframes && (!results || !payload)) || payload_stride < 16 || payload_stride % 16)
    return amod_ctx_fail(nullptr, "invalid argument", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lock(r->mu); // the memsets, the decode and the copies back, as one
  amod_group *g = r->g;
  std::vector<amod_shard> shards(r->sh.size());
  for (size_t k = 0; k < r->sh.size(); ++k) {
    ResidentShard &s = r->sh[k];
    if (s.nframes <= 0) continue;
    const size_t pb = (size_t)payload_stride * (size_t)s.nframes;
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess && s.payload_bytes < pb) {
      if (s.payload) (void)hipFree(s.payload);
      s.payload = nullptr;
      s.payload_bytes = 0;
      e = hipMalloc(&s.payload, pb);
      if (e == hipSuccess) s.payload_bytes = pb;
    }
    // the fast kernel writes only the decoded prefix of each slot: hand back zeros past it
    if (e == hipSuccess) e = hipMemsetAsync(s.payload, 0, pb, amod_ctx_stream(g->ctx[k]));
    if (e != hipSuccess) return amod_ctx_fail(nullptr, hipGetErrorString(e), AMOD_ERR_HIP);
    shards[k] = amod_shard{(const float *)s.samples, (const int64_t *)s.offsets, (const int32_t *)s.lengths,
                           (amod_result *)s.results, (uint8_t *)s.payload, payload_stride, nullptr, s.nframes, 0};
  }
  int rc = amod_group_decode_device(g, cfg, mode, shards.data(), options);
  if (rc != AMOD_SUCCESS) return rc;
  for (size_t k = 0; k < r->sh.size(); ++k) {
    const ResidentShard &s = r->sh[k];
    if (s.nframes <= 0) continue;
    hipStream_t st = amod_ctx_stream(g->ctx[k]);
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess)
      e = hipMemcpyAsync(results + s.first, s.results, sizeof(amod_result) * (size_t)s.nframes, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
      e = hipMemcpyAsync(payload + (size_t)s.first * (size_t)payload_stride, s.payload,
                         (size_t)payload_stride * (size_t)s.nframes, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return amod_ctx_fail(nullptr, hipGetErrorString(e), AMOD_ERR_HIP);
  }
  return amod_group_synchronize(g);
}
