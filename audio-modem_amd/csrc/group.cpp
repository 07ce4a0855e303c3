// group.cpp — one host process driving several GPUs (the Node host
// decoding one batch on N devices). A group holds one context per device; a batch is cut
// into contiguous frame ranges of about equal sample counts, each range decoded on its own
// device concurrently (host thread per device: H2D of the range's samples, the fast and
// exact kernels, D2H of its results straight into the caller's arrays). Frames are
// independent, so there is no device-to-device exchange on the data path.
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "amodem_internal.h"

struct amod_group {
  std::vector<amod_ctx *> ctx;
};

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
  // contiguous frame ranges of about equal sample counts
  std::vector<int64_t> cum((size_t)nframes + 1, 0);
  for (int32_t i = 0; i < nframes; ++i) cum[(size_t)i + 1] = cum[(size_t)i] + lengths[i];
  std::vector<int32_t> cut((size_t)nd + 1, 0);
  for (int k = 1; k < nd; ++k) {
    const int64_t want = cum.back() * k / nd;
    cut[(size_t)k] = (int32_t)(std::lower_bound(cum.begin(), cum.end(), want) - cum.begin());
    cut[(size_t)k] = std::max(cut[(size_t)k - 1], std::min(cut[(size_t)k], nframes));
  }
  cut[(size_t)nd] = nframes;
  std::vector<int> rc((size_t)nd, AMOD_SUCCESS);
  std::vector<std::string> err((size_t)nd);
  std::vector<std::thread> th;
  for (int k = 0; k < nd; ++k) {
    const int32_t a = cut[(size_t)k], b = cut[(size_t)k + 1];
    if (frames_per_device) frames_per_device[k] = b - a;
    if (b <= a) continue;
    th.emplace_back([&, k, a, b] {
      int64_t lo = INT64_MAX, hi = 0;
      for (int32_t i = a; i < b; ++i) { lo = std::min(lo, offsets[i]); hi = std::max(hi, offsets[i] + lengths[i]); }
      // keep every frame's offset mod 4: the fast path's block moments sit on 16-byte
      // boundaries of the buffer, so its approximate coarse_idx follows the alignment
      lo &= ~int64_t(3);
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
