// pipe.cpp — a depth-2 decode pipeline over two contexts of one device (amod_pipe_*).
//
// Consecutive device-resident batches (the bench's steps, a server's stream of batches)
// alternate between the two contexts, each decoding on a stream of the pipe's own, so
// batch i + 1's k_detect (the HBM-bound stream pass) starts while batch i's k_demod and
// frame ends are still running: the two kernels' tails and the dependent-launch gaps
// between them overlap (C2: 0.445 -> 0.42-0.43 ms per batch, C5 10 dB 1.60 -> 1.48-1.53,
// tools/pipeline_ab.py; the contexts' own streams or high-priority slot streams measured
// the same within the run-to-run spread).
//
// The caller works on the slot's stream (amod_pipe_next_stream: the stream the next decode
// runs on): it enqueues that batch's inputs there before the call and reads the results
// there after it, all in stream order, with no cross-stream event in the steady state. A
// caller that keeps its own stream passes it instead: the decode then starts once that
// stream reaches the call, and is joined onto it when the next decode is enqueued (or at
// amod_pipe_flush). That costs two cross-queue signals per batch, most of the overlap
// (C2 0.450 ms by hand on torch events; 0.53-0.55 ms when the caller's stream shared a
// hardware queue with a slot: GPU_MAX_HW_QUEUES is 4).
#include <hip/hip_runtime.h>

#include <string>

#include "amodem_internal.h"

struct amod_pipe {
  amod_ctx *ctx[2] = {nullptr, nullptr};
  hipStream_t slot[2] = {nullptr, nullptr}; // the streams the decodes run on
  hipEvent_t ev_in = nullptr;               // a caller's stream reached the call
  hipEvent_t ev_done[2] = {nullptr, nullptr};
  bool pending[2] = {false, false}; // decode on slot k not yet joined onto its caller's stream
  hipStream_t caller[2] = {nullptr, nullptr}; // the caller stream that issued slot k's pending decode
  int next = 0;
  int device = 0; // (close never touches the contexts: they may be closed already)
};

namespace {

int pipe_hip(amod_pipe *p, hipError_t e, const char *what) {
  const std::string msg = std::string(what) + ": " + hipGetErrorString(e);
  return amod_ctx_fail(p ? p->ctx[0] : nullptr, msg.c_str(), AMOD_ERR_HIP);
}
#define PIPE_TRY(p, x)                                 \
  do {                                                 \
    const hipError_t e_ = (x);                         \
    if (e_ != hipSuccess) return pipe_hip(p, e_, #x);  \
  } while (0)

} // namespace

extern "C" int amod_pipe_open(amod_ctx *a, amod_ctx *b, amod_pipe **out) {
  if (!out || !a || !b || a == b) return amod_ctx_fail(a, "amod_pipe_open: two distinct contexts", AMOD_ERR_ARG);
  if (amod_ctx_device(a) != amod_ctx_device(b))
    return amod_ctx_fail(a, "amod_pipe_open: the contexts are on different devices", AMOD_ERR_ARG);
  auto *p = new amod_pipe;
  p->ctx[0] = a;
  p->ctx[1] = b;
  p->device = amod_ctx_device(a);
  hipError_t e = hipSetDevice(p->device);
  for (int k = 0; k < 2 && e == hipSuccess; ++k) e = hipStreamCreateWithFlags(&p->slot[k], hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ev_in, hipEventDisableTiming);
  for (int k = 0; k < 2 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&p->ev_done[k], hipEventDisableTiming);
  if (e != hipSuccess) {
    const int rc = pipe_hip(p, e, "amod_pipe_open");
    amod_pipe_close(p);
    return rc;
  }
  *out = p;
  return AMOD_SUCCESS;
}

extern "C" int amod_pipe_close(amod_pipe *p) {
  if (!p) return AMOD_SUCCESS;
  (void)hipSetDevice(p->device);
  for (hipStream_t s : p->slot)
    if (s) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
  if (p->ev_in) (void)hipEventDestroy(p->ev_in);
  for (hipEvent_t e : p->ev_done)
    if (e) (void)hipEventDestroy(e);
  delete p; // (the contexts are the caller's)
  return AMOD_SUCCESS;
}

extern "C" void *amod_pipe_next_stream(const amod_pipe *p) { return p ? (void *)p->slot[p->next] : nullptr; }

extern "C" int amod_pipe_decode_device(amod_pipe *p, const amod_cfg *cfg, int32_t mode, const float *samples,
                                       const int64_t *offsets, const int32_t *lengths, int32_t nframes,
                                       amod_result *results, uint8_t *payload, int64_t payload_stride,
                                       uint32_t options, void *stream) {
  if (!p) return amod_ctx_fail(nullptr, "null pipe", AMOD_ERR_ARG);
  PIPE_TRY(p, hipSetDevice(p->device));
  const int k = p->next;
  amod_ctx *c = p->ctx[k];
  hipStream_t w = p->slot[k];
  hipStream_t s = (hipStream_t)stream;
  if (s == w) s = nullptr; // (the slot's own stream: plain stream order)
  if (s) { // this batch's inputs (and any use of slot k's previous results) are ordered before the call
    PIPE_TRY(p, hipEventRecord(p->ev_in, s));
    PIPE_TRY(p, hipStreamWaitEvent(w, p->ev_in, 0));
  }
  // Staggered slots: this decode starts once the other slot's latest k_detect is done, so
  // the detections (HBM-bound stream passes) run back to back and each k_demod runs beside
  // the next batch's detection. Unstaggered, both slots' k_detect ran at once, then both
  // k_demod: the overlap was only the kernels' tails and gaps
  if (amod_ctx_knobs(c)->pipe_stagger) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    PIPE_TRY(p, hipStreamIsCapturing(w, &cs));
    const hipEvent_t ev = amod_ctx_detect_event(p->ctx[k ^ 1]);
    if (ev && cs == hipStreamCaptureStatusNone) PIPE_TRY(p, hipStreamWaitEvent(w, ev, 0));
  }
  const int rc = amod_decode_device(c, cfg, mode, samples, offsets, lengths, nframes, results, payload,
                                    payload_stride, options, w);
  if (rc != AMOD_SUCCESS) {
    if (c != p->ctx[0]) amod_ctx_fail(p->ctx[0], amod_last_error(c), rc);
    return rc;
  }
  p->next = k ^ 1;
  if (s) {
    PIPE_TRY(p, hipEventRecord(p->ev_done[k], w));
    p->pending[k] = true;
    p->caller[k] = s;
  }
  // the previous decode (the other slot) is joined now, after this one's start was
  // recorded, onto the stream that issued it (whatever this call passed)
  if (p->pending[k ^ 1]) {
    PIPE_TRY(p, hipStreamWaitEvent(p->caller[k ^ 1], p->ev_done[k ^ 1], 0));
    p->pending[k ^ 1] = false;
  }
  return AMOD_SUCCESS;
}

extern "C" int amod_pipe_flush(amod_pipe *p, void *stream) {
  if (!p) return amod_ctx_fail(nullptr, "null pipe", AMOD_ERR_ARG);
  PIPE_TRY(p, hipSetDevice(p->device));
  if (!stream) { // slot-stream callers: their results are in stream order; a pending
                 // caller-stream decode is joined onto the stream that issued it
    for (int k = 0; k < 2; ++k)
      if (p->pending[k]) {
        PIPE_TRY(p, hipStreamWaitEvent(p->caller[k], p->ev_done[k], 0));
        p->pending[k] = false;
      }
    return AMOD_SUCCESS;
  }
  for (int k = 0; k < 2; ++k)
    if (p->pending[k]) { // onto the stream that issued it, and onto the one flushed
      PIPE_TRY(p, hipStreamWaitEvent(p->caller[k], p->ev_done[k], 0));
      if (p->caller[k] != (hipStream_t)stream) PIPE_TRY(p, hipStreamWaitEvent((hipStream_t)stream, p->ev_done[k], 0));
      p->pending[k] = false;
    }
  return AMOD_SUCCESS;
}

extern "C" int amod_pipe_synchronize(amod_pipe *p) {
  if (!p) return amod_ctx_fail(nullptr, "null pipe", AMOD_ERR_ARG);
  PIPE_TRY(p, hipSetDevice(p->device));
  for (hipStream_t s : p->slot) PIPE_TRY(p, hipStreamSynchronize(s));
  p->pending[0] = p->pending[1] = false;
  return AMOD_SUCCESS;
}
