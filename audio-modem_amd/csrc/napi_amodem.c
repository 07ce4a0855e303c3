/*
 * napi_amodem.c — N-API binding of libamodem (include/amodem.h) for Node.js.
 *
 * The thin C shim the JavaScript surface (audio-modem_amd/js/modem.js) calls:
 * plain typed arrays in, typed arrays out, no state beyond one lazily opened
 * amod_ctx per device. HIP failures throw Error(amod_last_error); per-frame
 * outcomes come back as amod_result records for the JS side to format with the
 * reference's exact strings (modem.js:557-654, 770-849).
 *
 *   decode(samples: Float32Array, offsets: Float64Array|null, lengths: Int32Array|null,
 *          cfg: object, mode: number, options: number, device?: number)
 *       -> { results: ArrayBuffer (96 B per frame), payload: ArrayBuffer, stride: number }
 *   decodeAsync(...same...) -> Promise of the same object (napi_async_work)
 *   loopback(samples, cfg, device?) -> analyzeLoopback receive core (status, preambleIdx,
 *          fineMetric, hRe, hIm, bytes)                            modem.js:975-1082
 *   crc32(Uint8Array) -> number                     modem.js:443-457
 *   preamble1(cfg) -> Float32Array                  modem.js:158-170
 *   txLegacy(cfg, data: Uint8Array, name: Uint8Array) -> Float32Array   modem.js:498-555
 *   txMeta(cfg, totalChunks, totalSize, chunkSize, name: Uint8Array)    modem.js:758
 *   txChunk(cfg, data: Uint8Array, seq)                                modem.js:763
 *   txTestSignal(cfg) -> Float32Array                                   modem.js:914-973
 *   estimateFrameSamples(cfg, payloadBytes) -> number                   modem.js:863-874
 *   numDataSubs(cfg) -> number, payloadStride(cfg, maxLen) -> number, abiVersion() -> number
 *   residentUpload(samples, offsets, lengths, cfg, ndevices) -> { handle, nframes, maxLen,
 *          framesPerDevice }: the batch made resident across GPUs 0 .. n-1 (amod_group_upload)
 *   residentDecodeAsync(handle, cfg, mode, options) -> Promise of { results, payload, stride }
 *          (amod_resident_decode: every GPU decodes its resident shard, no upload)
 *
 * cfg = { fft_size, cp_len, symbol_len, sample_rate, sub_start, sub_end,
 *         pilots: number[], modulation: 0|1|2, repetition }
 */
#define NAPI_VERSION 4
#include <node_api.h>

#include <execinfo.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "amodem.h"

#define MAX_DEVICES 16
static amod_ctx *g_ctx[MAX_DEVICES];
static amod_group *g_group[MAX_DEVICES + 1]; /* devices 0 .. n-1, opened on first use */

#define NAPI_TRY(env, call)                                                 \
  do {                                                                      \
    if ((call) != napi_ok) {                                                \
      const napi_extended_error_info *ei_ = NULL;                           \
      napi_get_last_error_info((env), &ei_);                                \
      bool pending_ = false;                                                \
      napi_is_exception_pending((env), &pending_);                          \
      if (!pending_)                                                        \
        napi_throw_error((env), NULL, ei_ && ei_->error_message ? ei_->error_message : "N-API call failed"); \
      return NULL;                                                          \
    }                                                                       \
  } while (0)

static napi_value throw_msg(napi_env env, const char *msg) {
  napi_throw_error(env, NULL, msg);
  return NULL;
}

static amod_ctx *get_ctx(napi_env env, int device) {
  if (device < 0 || device >= MAX_DEVICES) {
    napi_throw_range_error(env, NULL, "device index out of range");
    return NULL;
  }
  if (!g_ctx[device]) {
    amod_ctx *c = NULL;
    if (amod_open(device, &c) != AMOD_SUCCESS) {
      const char *e = amod_last_error(NULL);
      napi_throw_error(env, NULL, e && *e ? e : "amod_open failed");
      return NULL;
    }
    g_ctx[device] = c;
  }
  return g_ctx[device];
}

static int get_i32_prop(napi_env env, napi_value obj, const char *name, int32_t *out) {
  napi_value v;
  bool has = false;
  if (napi_has_named_property(env, obj, name, &has) != napi_ok || !has) return 0;
  if (napi_get_named_property(env, obj, name, &v) != napi_ok) return 0;
  return napi_get_value_int32(env, v, out) == napi_ok;
}

/* JS cfg object -> amod_cfg; throws TypeError and returns 0 on a malformed object */
static int to_cfg(napi_env env, napi_value obj, amod_cfg *c) {
  memset(c, 0, sizeof *c);
  static const char *names[] = {"fft_size", "cp_len", "symbol_len", "sample_rate", "sub_start", "sub_end",
                                "modulation", "repetition"};
  int32_t *dst[] = {&c->fft_size, &c->cp_len, &c->symbol_len, &c->sample_rate, &c->sub_start, &c->sub_end,
                    &c->modulation, &c->repetition};
  for (int i = 0; i < 8; ++i)
    if (!get_i32_prop(env, obj, names[i], dst[i])) {
      char msg[96];
      snprintf(msg, sizeof msg, "cfg.%s missing or not a number", names[i]);
      napi_throw_type_error(env, NULL, msg);
      return 0;
    }
  napi_value pil;
  bool is_arr = false;
  uint32_t n = 0;
  if (napi_get_named_property(env, obj, "pilots", &pil) != napi_ok || napi_is_array(env, pil, &is_arr) != napi_ok ||
      !is_arr || napi_get_array_length(env, pil, &n) != napi_ok || n > AMOD_MAX_PILOTS) {
    napi_throw_type_error(env, NULL, "cfg.pilots must be an array of at most 32 numbers");
    return 0;
  }
  c->npilots = (int32_t)n;
  for (uint32_t i = 0; i < n; ++i) {
    napi_value e;
    if (napi_get_element(env, pil, i, &e) != napi_ok || napi_get_value_int32(env, e, &c->pilots[i]) != napi_ok) {
      napi_throw_type_error(env, NULL, "cfg.pilots must be an array of numbers");
      return 0;
    }
  }
  return 1;
}

/* typed array view: data pointer + element count, checks the element type */
static int typed(napi_env env, napi_value v, napi_typedarray_type want, void **data, size_t *len) {
  bool is = false;
  if (napi_is_typedarray(env, v, &is) != napi_ok || !is) return 0;
  napi_typedarray_type t;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, len, data, &ab, &off) != napi_ok) return 0;
  return t == want;
}

static int is_nullish(napi_env env, napi_value v) {
  napi_valuetype t;
  return napi_typeof(env, v, &t) == napi_ok && (t == napi_null || t == napi_undefined);
}

/* the group of GPUs 0 .. n-1, opened on first use (AMODEM_GROUP_DEVICES="0,0": the device
   list to use instead, tests on one GPU); throws and returns NULL on failure */
static amod_group *get_group(napi_env env, int32_t ndev) {
  if (ndev < 1 || ndev > MAX_DEVICES) {
    napi_throw_range_error(env, NULL, "devices out of range");
    return NULL;
  }
  if (!g_group[ndev]) {
    int32_t ids[MAX_DEVICES];
    for (int32_t i = 0; i < ndev; ++i) ids[i] = i;
    const char *lst = getenv("AMODEM_GROUP_DEVICES");
    for (int32_t i = 0; lst && *lst && i < ndev; ++i) {
      ids[i] = (int32_t)strtol(lst, (char **)&lst, 10);
      if (*lst == ',') ++lst;
    }
    if (amod_group_open(ids, ndev, &g_group[ndev]) != AMOD_SUCCESS) {
      throw_msg(env, amod_last_error(NULL));
      return NULL;
    }
  }
  return g_group[ndev];
}

/* A resident batch holds GPU memory, so it is released explicitly (DeviceBatch.free() ->
   residentFree), or at the environment's cleanup, and its JS handle is a plain number,
   not a napi external: Node 12 gives every external a self-deleting weak reference, even
   without a finalizer, and a GC at exit ran its second-pass phantom callback after the
   environment was torn down (SIGSEGV inside libnode after the script's output,
   tools/node_c4.py). busy counts decodes in flight: a free() during one takes effect
   when the last completes. Main thread only. */
typedef struct resident_box {
  amod_resident *r;
  int32_t nframes, max_len;
  int32_t busy, free_pending;
  int64_t id;
  struct resident_box *next;
} resident_box;
static resident_box *g_boxes = NULL; /* the live boxes of this environment */
static int64_t g_box_next = 1;

static resident_box *resident_find(napi_env env, napi_value h) {
  int64_t id = 0;
  if (napi_get_value_int64(env, h, &id) != napi_ok) return NULL;
  for (resident_box *b = g_boxes; b; b = b->next)
    if (b->id == id) return b;
  return NULL;
}
static void resident_release(resident_box *b) {
  if (b->busy) {
    b->free_pending = 1;
    return;
  }
  amod_resident_free(b->r);
  for (resident_box **pp = &g_boxes; *pp; pp = &(*pp)->next)
    if (*pp == b) {
      *pp = b->next;
      break;
    }
  free(b);
}
static void resident_cleanup(void *arg) {
  (void)arg;
  while (g_boxes) {
    resident_box *b = g_boxes;
    g_boxes = b->next;
    amod_resident_free(b->r);
    free(b);
  }
}


/* ------------------------------------------------------------------ decode */
typedef struct {
  amod_ctx *ctx;
  amod_cfg cfg;
  amod_group *group; /* decodeBatch(..., {devices: n > 1}): the batch split across n GPUs */
  amod_resident *resident; /* residentDecodeAsync: a batch already resident on the GPUs */
  struct resident_box *box; /* (its box: busy while this decode runs) */
  int32_t mode, nframes;
  uint32_t options;
  const float *samples;
  int64_t nsamples;
  int64_t *offsets;
  int32_t *lengths;
  int64_t stride;
  void *results, *payload; /* ArrayBuffer backing stores (owned by JS objects) */
  int rc;
  double native_ms; /* wall time of the library call (run_decode), for the bench's split */
  napi_threadsafe_function progress; /* decodeAsync's onFrames(done, results, payload, stride) */
  char err[256];
  /* async only */
  napi_ref refs[3];
  napi_value res_ab, pay_ab;
  napi_ref res_ref, pay_ref;
  napi_deferred deferred;
  napi_async_work work;
} decode_job;

/* parse args into a job; allocates offsets/lengths and the output ArrayBuffers */
static int prepare(napi_env env, napi_callback_info info, decode_job *j, napi_value argv_out[3]) {
  size_t argc = 8;
  napi_value argv[8];
  memset(j, 0, sizeof *j);
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 6) {
    napi_throw_type_error(env, NULL, "decode(samples, offsets, lengths, cfg, mode, options[, device[, ndevices]])");
    return 0;
  }
  void *sp;
  size_t ns;
  if (!typed(env, argv[0], napi_float32_array, &sp, &ns)) {
    napi_throw_type_error(env, NULL, "samples must be a Float32Array");
    return 0;
  }
  j->samples = (const float *)sp;
  j->nsamples = (int64_t)ns;
  if (!to_cfg(env, argv[3], &j->cfg)) return 0;
  if (napi_get_value_int32(env, argv[4], &j->mode) != napi_ok) {
    napi_throw_type_error(env, NULL, "mode must be a number");
    return 0;
  }
  if (napi_get_value_uint32(env, argv[5], &j->options) != napi_ok) j->options = 0;
  int32_t device = 0;
  if (argc >= 7 && !is_nullish(env, argv[6]) && napi_get_value_int32(env, argv[6], &device) != napi_ok) device = 0;
  int32_t ndev = 1;
  if (argc >= 8 && !is_nullish(env, argv[7]) && napi_get_value_int32(env, argv[7], &ndev) != napi_ok) ndev = 1;
  if (ndev > 1) {
    j->group = get_group(env, ndev);
    if (!j->group) return 0;
  } else {
    j->ctx = get_ctx(env, device);
    if (!j->ctx) return 0;
  }

  if (is_nullish(env, argv[1])) { /* one frame: the whole buffer */
    j->nframes = 1;
    j->offsets = (int64_t *)calloc(1, sizeof(int64_t));
    j->lengths = (int32_t *)calloc(1, sizeof(int32_t));
    if (!j->offsets || !j->lengths) return throw_msg(env, "out of memory"), 0;
    if (ns > INT32_MAX) return napi_throw_range_error(env, NULL, "frame longer than 2^31-1 samples"), 0;
    j->lengths[0] = (int32_t)ns;
  } else {
    void *op, *lp;
    size_t no, nl;
    if (!typed(env, argv[1], napi_float64_array, &op, &no) || !typed(env, argv[2], napi_int32_array, &lp, &nl) ||
        no != nl || no > INT32_MAX) {
      napi_throw_type_error(env, NULL, "offsets must be a Float64Array and lengths an Int32Array of equal length");
      return 0;
    }
    j->nframes = (int32_t)no;
    j->offsets = (int64_t *)malloc(sizeof(int64_t) * (no ? no : 1));
    j->lengths = (int32_t *)malloc(sizeof(int32_t) * (no ? no : 1));
    if (!j->offsets || !j->lengths) return throw_msg(env, "out of memory"), 0;
    const double *od = (const double *)op;
    const int32_t *ld = (const int32_t *)lp;
    for (size_t i = 0; i < no; ++i) {
      const double o = od[i];
      if (!(o >= 0) || o != (double)(int64_t)o || ld[i] < 0 || (int64_t)o + ld[i] > (int64_t)ns) {
        napi_throw_range_error(env, NULL, "frame slice outside the sample buffer");
        return 0;
      }
      j->offsets[i] = (int64_t)o;
      j->lengths[i] = ld[i];
    }
  }
  int32_t maxlen = 0;
  for (int32_t i = 0; i < j->nframes; ++i) maxlen = j->lengths[i] > maxlen ? j->lengths[i] : maxlen;
  j->stride = amod_payload_stride(&j->cfg, maxlen);
  if (j->stride <= 0) {
    napi_throw_type_error(env, NULL, "invalid OFDM configuration");
    return 0;
  }
  if (napi_create_arraybuffer(env, (size_t)j->nframes * sizeof(amod_result), &j->results, &j->res_ab) != napi_ok ||
      napi_create_arraybuffer(env, (size_t)j->nframes * (size_t)j->stride, &j->payload, &j->pay_ab) != napi_ok) {
    napi_throw_error(env, NULL, "cannot allocate decode outputs");
    return 0;
  }
  // (no memset: napi_create_arraybuffer's memory is zero-filled already, and touching the
  // payload's pages here, on the JS thread, cost every batch a pass over 68 MB on C4; the
  // slots past each frame's decoded bytes must read as zero)
  argv_out[0] = argv[0];
  argv_out[1] = argv[1];
  argv_out[2] = argv[2];
  return 1;
}

/* onFrames: called on the JS thread, in order, whenever records [0, done) are in the
 * results/payload buffers (amod_decode_host_progress), so the caller formats those frames
 * while the library decodes the rest. The call context outlives the decode job: queued
 * calls may run after the promise settled (the finalizer frees it) */
typedef struct {
  napi_ref res_ref, pay_ref;
  double stride;
} progress_ctx;

static void progress_call_js(napi_env env, napi_value cb, void *context, void *data) {
  progress_ctx *pc = (progress_ctx *)context;
  if (!env || !cb) return;
  napi_value argv[4], undef;
  if (napi_create_int32(env, (int32_t)(intptr_t)data, &argv[0]) != napi_ok ||
      napi_get_reference_value(env, pc->res_ref, &argv[1]) != napi_ok ||
      napi_get_reference_value(env, pc->pay_ref, &argv[2]) != napi_ok ||
      napi_create_double(env, pc->stride, &argv[3]) != napi_ok || napi_get_undefined(env, &undef) != napi_ok)
    return;
  /* modem.js's onFrames keeps any error of its own for the promise; should a callback
   * throw anyway, the exception is cleared here (a threadsafe-function call has no caller
   * to propagate it to, and left pending it would end the process) */
  if (napi_call_function(env, undef, cb, 4, argv, NULL) == napi_pending_exception) {
    napi_value exc;
    napi_get_and_clear_last_exception(env, &exc);
  }
}

static void progress_finalize(napi_env env, void *data, void *hint) {
  (void)hint;
  progress_ctx *pc = (progress_ctx *)data;
  napi_delete_reference(env, pc->res_ref);
  napi_delete_reference(env, pc->pay_ref);
  free(pc);
}

static void progress_native(void *user, int32_t done) {
  napi_call_threadsafe_function((napi_threadsafe_function)user, (void *)(intptr_t)done, napi_tsfn_nonblocking);
}

static void run_decode(decode_job *j) {
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  if (j->resident)
    j->rc = amod_resident_decode(j->resident, &j->cfg, j->mode, j->options, (amod_result *)j->results,
                                 (uint8_t *)j->payload, j->stride);
  else if (j->group)
    j->rc = amod_group_decode_host(j->group, &j->cfg, j->mode, j->samples, j->nsamples, j->offsets, j->lengths,
                                   j->nframes, (amod_result *)j->results, (uint8_t *)j->payload, j->stride, j->options,
                                   NULL);
  else if (j->progress)
    j->rc = amod_decode_host_progress(j->ctx, &j->cfg, j->mode, j->samples, j->nsamples, j->offsets, j->lengths,
                                      j->nframes, (amod_result *)j->results, (uint8_t *)j->payload, j->stride,
                                      j->options, progress_native, (void *)j->progress);
  else
    j->rc = amod_decode_host(j->ctx, &j->cfg, j->mode, j->samples, j->nsamples, j->offsets, j->lengths, j->nframes,
                             (amod_result *)j->results, (uint8_t *)j->payload, j->stride, j->options);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  j->native_ms = (double)(t1.tv_sec - t0.tv_sec) * 1e3 + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-6;
  if (j->rc != AMOD_SUCCESS) {
    const char *e = amod_last_error(j->group || j->resident ? NULL : j->ctx);
    snprintf(j->err, sizeof j->err, "libamodem error %d: %s", j->rc, e ? e : "");
  }
}

static napi_value result_object(napi_env env, decode_job *j, napi_value res_ab, napi_value pay_ab) {
  napi_value out, st;
  NAPI_TRY(env, napi_create_object(env, &out));
  NAPI_TRY(env, napi_set_named_property(env, out, "results", res_ab));
  NAPI_TRY(env, napi_set_named_property(env, out, "payload", pay_ab));
  NAPI_TRY(env, napi_create_double(env, (double)j->stride, &st));
  NAPI_TRY(env, napi_set_named_property(env, out, "stride", st));
  NAPI_TRY(env, napi_create_double(env, j->native_ms, &st));
  NAPI_TRY(env, napi_set_named_property(env, out, "nativeMs", st));
  return out;
}

static void free_job(decode_job *j) {
  free(j->offsets);
  free(j->lengths);
  j->offsets = NULL;
  j->lengths = NULL;
}

static napi_value js_decode(napi_env env, napi_callback_info info) {
  decode_job j;
  napi_value keep[3];
  if (!prepare(env, info, &j, keep)) {
    free_job(&j);
    return NULL;
  }
  run_decode(&j);
  free_job(&j);
  if (j.rc != AMOD_SUCCESS) return throw_msg(env, j.err);
  return result_object(env, &j, j.res_ab, j.pay_ab);
}

static void async_execute(napi_env env, void *data) {
  (void)env;
  run_decode((decode_job *)data);
}

static void async_complete(napi_env env, napi_status status, void *data) {
  decode_job *j = (decode_job *)data;
  napi_value res_ab, pay_ab, val;
  napi_get_reference_value(env, j->res_ref, &res_ab);
  napi_get_reference_value(env, j->pay_ref, &pay_ab);
  if (status != napi_ok || j->rc != AMOD_SUCCESS) {
    napi_value msg, err;
    napi_create_string_utf8(env, j->rc != AMOD_SUCCESS ? j->err : "decode cancelled", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, j->deferred, err);
  } else {
    val = result_object(env, j, res_ab, pay_ab);
    napi_resolve_deferred(env, j->deferred, val);
  }
  for (int i = 0; i < 3; ++i)
    if (j->refs[i]) napi_delete_reference(env, j->refs[i]);
  napi_delete_reference(env, j->res_ref);
  napi_delete_reference(env, j->pay_ref);
  napi_delete_async_work(env, j->work);
  if (j->progress) napi_release_threadsafe_function(j->progress, napi_tsfn_release);
  if (j->box && --j->box->busy == 0 && j->box->free_pending) resident_release(j->box);
  free_job(j);
  free(j);
}

/* a job whose promise was never created: drop its references and memory */
static void async_discard(napi_env env, decode_job *j) {
  for (int i = 0; i < 3; ++i)
    if (j->refs[i]) napi_delete_reference(env, j->refs[i]);
  napi_delete_reference(env, j->res_ref);
  napi_delete_reference(env, j->pay_ref);
  free_job(j);
  free(j);
}

static napi_value js_decode_async(napi_env env, napi_callback_info info) {
  decode_job *j = (decode_job *)malloc(sizeof *j);
  if (!j) return throw_msg(env, "out of memory");
  napi_value keep[3];
  if (!prepare(env, info, j, keep)) {
    free_job(j);
    free(j);
    return NULL;
  }
  /* keep the caller's typed arrays (samples + offsets/lengths) and the outputs alive */
  for (int i = 0; i < 3; ++i) {
    napi_valuetype t;
    napi_typeof(env, keep[i], &t);
    if (t == napi_object) napi_create_reference(env, keep[i], 1, &j->refs[i]);
  }
  napi_create_reference(env, j->res_ab, 1, &j->res_ref);
  napi_create_reference(env, j->pay_ab, 1, &j->pay_ref);
  napi_value promise, name;
  NAPI_TRY(env, napi_create_string_utf8(env, "amodem.decode", NAPI_AUTO_LENGTH, &name));
  { /* optional 9th argument: onFrames (single-device host decodes) */
    size_t argc = 9;
    napi_value argv[9];
    napi_valuetype t = napi_undefined;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) == napi_ok && argc >= 9) napi_typeof(env, argv[8], &t);
    if (t == napi_function && j->ctx) {
      progress_ctx *pc = (progress_ctx *)calloc(1, sizeof *pc);
      if (!pc) {
        async_discard(env, j);
        return throw_msg(env, "out of memory");
      }
      pc->stride = (double)j->stride;
      napi_create_reference(env, j->res_ab, 1, &pc->res_ref);
      napi_create_reference(env, j->pay_ab, 1, &pc->pay_ref);
      if (napi_create_threadsafe_function(env, argv[8], NULL, name, 0, 1, pc, progress_finalize, pc, progress_call_js,
                                          &j->progress) != napi_ok) {
        progress_finalize(env, pc, NULL);
        async_discard(env, j);
        return throw_msg(env, "cannot create the progress callback");
      }
    }
  }
  NAPI_TRY(env, napi_create_promise(env, &j->deferred, &promise));
  NAPI_TRY(env, napi_create_async_work(env, NULL, name, async_execute, async_complete, j, &j->work));
  NAPI_TRY(env, napi_queue_async_work(env, j->work));
  return promise;
}

/* ------------------------------------------------------- resident batches */
static napi_value js_resident_upload(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 5)
    return napi_throw_type_error(env, NULL, "residentUpload(samples, offsets, lengths, cfg, ndevices)"), NULL;
  void *sp, *op, *lp;
  size_t ns, no, nl;
  if (!typed(env, argv[0], napi_float32_array, &sp, &ns) || !typed(env, argv[1], napi_float64_array, &op, &no) ||
      !typed(env, argv[2], napi_int32_array, &lp, &nl) || no != nl || no > INT32_MAX)
    return napi_throw_type_error(env, NULL, "samples: Float32Array, offsets: Float64Array, lengths: Int32Array"), NULL;
  amod_cfg cfg;
  if (!to_cfg(env, argv[3], &cfg)) return NULL;
  int32_t ndev = 1;
  if (napi_get_value_int32(env, argv[4], &ndev) != napi_ok) ndev = 1;
  amod_group *g = get_group(env, ndev);
  if (!g) return NULL;
  int64_t *offs = (int64_t *)malloc(sizeof(int64_t) * (no ? no : 1));
  if (!offs) return throw_msg(env, "out of memory");
  const double *od = (const double *)op;
  const int32_t *ld = (const int32_t *)lp;
  int32_t max_len = 0;
  for (size_t i = 0; i < no; ++i) {
    if (!(od[i] >= 0) || od[i] != (double)(int64_t)od[i] || ld[i] < 0 || (int64_t)od[i] + ld[i] > (int64_t)ns) {
      free(offs);
      return napi_throw_range_error(env, NULL, "frame slice outside the sample buffer"), NULL;
    }
    offs[i] = (int64_t)od[i];
    if (ld[i] > max_len) max_len = ld[i];
  }
  resident_box *b = (resident_box *)calloc(1, sizeof *b);
  if (!b) {
    free(offs);
    return throw_msg(env, "out of memory");
  }
  const int rc = amod_group_upload(g, &cfg, (const float *)sp, (int64_t)ns, offs, ld, (int32_t)no, &b->r);
  free(offs);
  if (rc != AMOD_SUCCESS) {
    free(b);
    return throw_msg(env, amod_last_error(NULL));
  }
  b->nframes = (int32_t)no;
  b->max_len = max_len;
  static int hooked = 0;
  if (!hooked) {
    napi_add_env_cleanup_hook(env, resident_cleanup, NULL);
    hooked = 1;
  }
  b->id = g_box_next++;
  b->next = g_boxes;
  g_boxes = b;
  napi_value out, h, v, arr;
  NAPI_TRY(env, napi_create_int64(env, b->id, &h));
  NAPI_TRY(env, napi_create_object(env, &out));
  NAPI_TRY(env, napi_set_named_property(env, out, "handle", h));
  NAPI_TRY(env, napi_create_int32(env, b->nframes, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "nframes", v));
  NAPI_TRY(env, napi_create_int32(env, max_len, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "maxLen", v));
  int32_t per[MAX_DEVICES];
  amod_resident_frames(b->r, per);
  NAPI_TRY(env, napi_create_array_with_length(env, (size_t)ndev, &arr));
  for (int32_t k = 0; k < ndev; ++k) {
    NAPI_TRY(env, napi_create_int32(env, per[k], &v));
    NAPI_TRY(env, napi_set_element(env, arr, (uint32_t)k, v));
  }
  NAPI_TRY(env, napi_set_named_property(env, out, "framesPerDevice", arr));
  return out;
}

static napi_value js_resident_decode_async(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 4)
    return napi_throw_type_error(env, NULL, "residentDecodeAsync(handle, cfg, mode, options)"), NULL;
  resident_box *b = resident_find(env, argv[0]);
  if (!b || b->free_pending) return throw_msg(env, "the resident batch was freed (or never uploaded)");
  decode_job *j = (decode_job *)calloc(1, sizeof *j);
  if (!j) return throw_msg(env, "out of memory");
  if (!to_cfg(env, argv[1], &j->cfg)) {
    free(j);
    return NULL;
  }
  if (napi_get_value_int32(env, argv[2], &j->mode) != napi_ok) {
    free(j);
    return napi_throw_type_error(env, NULL, "mode must be a number"), NULL;
  }
  if (napi_get_value_uint32(env, argv[3], &j->options) != napi_ok) j->options = 0;
  j->resident = b->r;
  j->box = b;
  ++b->busy;
  j->nframes = b->nframes;
  j->stride = amod_payload_stride(&j->cfg, b->max_len);
  if (napi_create_arraybuffer(env, (size_t)j->nframes * sizeof(amod_result), &j->results, &j->res_ab) != napi_ok ||
      napi_create_arraybuffer(env, (size_t)j->nframes * (size_t)j->stride, &j->payload, &j->pay_ab) != napi_ok) {
    free(j);
    return throw_msg(env, "cannot allocate decode outputs");
  }
  /* keep the handle (and so the resident batch) alive until the decode completes */
  napi_create_reference(env, argv[0], 1, &j->refs[0]);
  napi_create_reference(env, j->res_ab, 1, &j->res_ref);
  napi_create_reference(env, j->pay_ab, 1, &j->pay_ref);
  napi_value promise, name;
  NAPI_TRY(env, napi_create_promise(env, &j->deferred, &promise));
  NAPI_TRY(env, napi_create_string_utf8(env, "amodem.residentDecode", NAPI_AUTO_LENGTH, &name));
  NAPI_TRY(env, napi_create_async_work(env, NULL, name, async_execute, async_complete, j, &j->work));
  NAPI_TRY(env, napi_queue_async_work(env, j->work));
  return promise;
}

/* residentFree(handle): the batch's GPU memory released now (after a decode in flight) */
static napi_value js_resident_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 1)
    return napi_throw_type_error(env, NULL, "residentFree(handle from residentUpload)"), NULL;
  resident_box *b = resident_find(env, argv[0]);
  if (b && !b->free_pending) resident_release(b); /* (a second free() is a no-op) */
  return NULL;
}

/* loopback(samples: Float32Array, cfg, device?) -> { status, preambleIdx, fineMetric,
     hRe: Float64Array, hIm: Float64Array, bytes: Uint8Array }   (modem.js:975-1082 core) */
static napi_value js_loopback(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 2)
    return napi_throw_type_error(env, NULL, "loopback(samples, cfg[, device])"), NULL;
  void *sp;
  size_t ns;
  if (!typed(env, argv[0], napi_float32_array, &sp, &ns) || ns > INT32_MAX)
    return napi_throw_type_error(env, NULL, "samples must be a Float32Array"), NULL;
  amod_cfg c;
  if (!to_cfg(env, argv[1], &c)) return NULL;
  int32_t device = 0;
  if (argc >= 3 && !is_nullish(env, argv[2])) napi_get_value_int32(env, argv[2], &device);
  amod_ctx *ctx = get_ctx(env, device);
  if (!ctx) return NULL;
  amod_result res;
  amod_debug *dbg = (amod_debug *)calloc(1, sizeof(amod_debug));
  const int64_t cap = amod_payload_stride(&c, (int64_t)ns);
  uint8_t *bytes = (uint8_t *)calloc(1, (size_t)(cap > 0 ? cap : 1));
  if (!dbg || !bytes) { free(dbg); free(bytes); return throw_msg(env, "out of memory"); }
  const int rc = amod_analyze_loopback(ctx, &c, (const float *)sp, (int64_t)ns, &res, dbg, bytes, cap);
  if (rc != AMOD_SUCCESS) {
    char msg[256];
    const char *e = amod_last_error(ctx);
    snprintf(msg, sizeof msg, "libamodem error %d: %s", rc, e ? e : "");
    free(dbg); free(bytes);
    return throw_msg(env, msg);
  }
  const int nband = c.sub_end - c.sub_start + 1;
  napi_value out, v, ab, ta;
  void *p;
  NAPI_TRY(env, napi_create_object(env, &out));
  NAPI_TRY(env, napi_create_int32(env, res.status, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "status", v));
  NAPI_TRY(env, napi_create_int32(env, res.preamble_idx, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "preambleIdx", v));
  NAPI_TRY(env, napi_create_double(env, dbg->fine_metric, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "fineMetric", v));
  const double *src[2] = {dbg->h_re, dbg->h_im};
  const char *names[2] = {"hRe", "hIm"};
  for (int k = 0; k < 2; ++k) {
    NAPI_TRY(env, napi_create_arraybuffer(env, sizeof(double) * (size_t)nband, &p, &ab));
    memcpy(p, src[k], sizeof(double) * (size_t)nband);
    NAPI_TRY(env, napi_create_typedarray(env, napi_float64_array, (size_t)nband, ab, 0, &ta));
    NAPI_TRY(env, napi_set_named_property(env, out, names[k], ta));
  }
  const int64_t nb = res.status == AMOD_OK ? (res.nbytes < cap ? res.nbytes : cap) : 0;
  NAPI_TRY(env, napi_create_arraybuffer(env, (size_t)nb, &p, &ab));
  if (nb) memcpy(p, bytes, (size_t)nb);
  NAPI_TRY(env, napi_create_typedarray(env, napi_uint8_array, (size_t)nb, ab, 0, &ta));
  NAPI_TRY(env, napi_set_named_property(env, out, "bytes", ta));
  free(dbg);
  free(bytes);
  return out;
}

/* ------------------------------------------------------------ host utilities */
static napi_value make_f32(napi_env env, int64_t n, float **data) {
  napi_value ab, ta;
  void *p;
  NAPI_TRY(env, napi_create_arraybuffer(env, (size_t)(n > 0 ? n : 0) * sizeof(float), &p, &ab));
  NAPI_TRY(env, napi_create_typedarray(env, napi_float32_array, (size_t)(n > 0 ? n : 0), ab, 0, &ta));
  *data = (float *)p;
  return ta;
}

static int get_args(napi_env env, napi_callback_info info, size_t want, napi_value *argv) {
  size_t argc = want;
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < want) {
    napi_throw_type_error(env, NULL, "wrong number of arguments");
    return 0;
  }
  return 1;
}

static int get_u8(napi_env env, napi_value v, const uint8_t **p, int32_t *n) {
  void *d;
  size_t len;
  if (!typed(env, v, napi_uint8_array, &d, &len) || len > INT32_MAX) {
    napi_throw_type_error(env, NULL, "expected a Uint8Array");
    return 0;
  }
  *p = (const uint8_t *)d;
  *n = (int32_t)len;
  return 1;
}

static napi_value js_crc32(napi_env env, napi_callback_info info) {
  napi_value argv[1], out;
  if (!get_args(env, info, 1, argv)) return NULL;
  const uint8_t *p;
  int32_t n;
  if (!get_u8(env, argv[0], &p, &n)) return NULL;
  NAPI_TRY(env, napi_create_uint32(env, amod_crc32(p, (size_t)n), &out));
  return out;
}

static napi_value js_preamble1(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  amod_cfg c;
  if (!get_args(env, info, 1, argv) || !to_cfg(env, argv[0], &c)) return NULL;
  float *d;
  napi_value ta = make_f32(env, c.symbol_len, &d);
  if (!ta) return NULL;
  if (amod_preamble1(&c, d) != AMOD_SUCCESS) return throw_msg(env, "invalid OFDM configuration");
  return ta;
}

static napi_value js_tx_legacy(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  amod_cfg c;
  const uint8_t *data, *name;
  int32_t nd, nn;
  if (!get_args(env, info, 3, argv) || !to_cfg(env, argv[0], &c) || !get_u8(env, argv[1], &data, &nd) ||
      !get_u8(env, argv[2], &name, &nn))
    return NULL;
  const int64_t n = amod_tx_legacy(&c, data, nd, name, nn, NULL);
  if (n < 0) return throw_msg(env, "invalid transmit arguments");
  float *d;
  napi_value ta = make_f32(env, n, &d);
  if (ta && n) amod_tx_legacy(&c, data, nd, name, nn, d);
  return ta;
}

static napi_value js_tx_meta(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  amod_cfg c;
  int32_t tc, ts, cs, nn;
  const uint8_t *name;
  if (!get_args(env, info, 5, argv) || !to_cfg(env, argv[0], &c)) return NULL;
  if (napi_get_value_int32(env, argv[1], &tc) != napi_ok || napi_get_value_int32(env, argv[2], &ts) != napi_ok ||
      napi_get_value_int32(env, argv[3], &cs) != napi_ok)
    return napi_throw_type_error(env, NULL, "totalChunks/totalFileSize/chunkSize must be numbers"), NULL;
  if (!get_u8(env, argv[4], &name, &nn)) return NULL;
  const int64_t n = amod_tx_meta(&c, tc, ts, cs, name, nn, NULL);
  if (n < 0) return throw_msg(env, "invalid transmit arguments");
  float *d;
  napi_value ta = make_f32(env, n, &d);
  if (ta && n) amod_tx_meta(&c, tc, ts, cs, name, nn, d);
  return ta;
}

static napi_value js_tx_chunk(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  amod_cfg c;
  const uint8_t *data;
  int32_t nd, seq;
  if (!get_args(env, info, 3, argv) || !to_cfg(env, argv[0], &c) || !get_u8(env, argv[1], &data, &nd)) return NULL;
  if (napi_get_value_int32(env, argv[2], &seq) != napi_ok)
    return napi_throw_type_error(env, NULL, "seqNum must be a number"), NULL;
  const int64_t n = amod_tx_chunk(&c, data, nd, seq, NULL);
  if (n < 0) return throw_msg(env, "invalid transmit arguments");
  float *d;
  napi_value ta = make_f32(env, n, &d);
  if (ta && n) amod_tx_chunk(&c, data, nd, seq, d);
  return ta;
}

static napi_value js_tx_test(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  amod_cfg c;
  if (!get_args(env, info, 1, argv) || !to_cfg(env, argv[0], &c)) return NULL;
  const int64_t n = amod_tx_test_signal(&c, NULL);
  if (n < 0) return throw_msg(env, "invalid transmit arguments");
  float *d;
  napi_value ta = make_f32(env, n, &d);
  if (ta && n) amod_tx_test_signal(&c, d);
  return ta;
}

static napi_value js_estimate(napi_env env, napi_callback_info info) {
  napi_value argv[2], out;
  amod_cfg c;
  int32_t nb;
  if (!get_args(env, info, 2, argv) || !to_cfg(env, argv[0], &c)) return NULL;
  if (napi_get_value_int32(env, argv[1], &nb) != napi_ok)
    return napi_throw_type_error(env, NULL, "payloadBytes must be a number"), NULL;
  NAPI_TRY(env, napi_create_int32(env, amod_estimate_frame_samples(&c, nb), &out));
  return out;
}

static napi_value js_num_data_subs(napi_env env, napi_callback_info info) {
  napi_value argv[1], out;
  amod_cfg c;
  if (!get_args(env, info, 1, argv) || !to_cfg(env, argv[0], &c)) return NULL;
  NAPI_TRY(env, napi_create_int32(env, amod_num_data_subs(&c), &out));
  return out;
}

static napi_value js_payload_stride(napi_env env, napi_callback_info info) {
  napi_value argv[2], out;
  amod_cfg c;
  int64_t ml;
  if (!get_args(env, info, 2, argv) || !to_cfg(env, argv[0], &c)) return NULL;
  if (napi_get_value_int64(env, argv[1], &ml) != napi_ok)
    return napi_throw_type_error(env, NULL, "maxLen must be a number"), NULL;
  NAPI_TRY(env, napi_create_double(env, (double)amod_payload_stride(&c, ml), &out));
  return out;
}

static napi_value js_abi(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value out;
  NAPI_TRY(env, napi_create_int32(env, amod_abi_version(), &out));
  return out;
}


/* ----------------------------------------------- chunk assembler / stream receive */
/* Assemblers and live receivers get numeric handles for the reason resident batches do
   (no napi externals: their weak references crash Node 12 at exit). Each is released by
   close() or at the environment's cleanup, live receivers before assemblers. A live
   receiver uses its assembler: closing the assembler first takes effect when the last
   receiver on it closes. Main thread only. */
enum { OBJ_ASM = 1, OBJ_LIVE = 2 };
typedef struct obj_box {
  int32_t kind;
  int32_t users;        /* OBJ_ASM: live receivers open on it */
  int32_t close_pending;
  int64_t id;
  void *p;
  struct obj_box *dep;  /* OBJ_LIVE: its assembler's box */
  struct obj_box *next;
} obj_box;
static obj_box *g_objs = NULL;
static int64_t g_obj_next = 1;

static void obj_unlink_free(obj_box *b) {
  for (obj_box **pp = &g_objs; *pp; pp = &(*pp)->next)
    if (*pp == b) {
      *pp = b->next;
      break;
    }
  free(b);
}
static void obj_release(obj_box *b) {
  if (b->kind == OBJ_ASM) {
    if (b->users) {
      b->close_pending = 1;
      return;
    }
    amod_asm_close((amod_assembler *)b->p);
    obj_unlink_free(b);
    return;
  }
  amod_live_close((amod_live *)b->p);
  obj_box *a = b->dep;
  obj_unlink_free(b);
  if (a && --a->users == 0 && a->close_pending) obj_release(a);
}
static void obj_cleanup(void *arg) {
  (void)arg;
  for (int kind = OBJ_LIVE; kind >= OBJ_ASM; --kind) {
    obj_box **pp = &g_objs;
    while (*pp) {
      obj_box *b = *pp;
      if (b->kind != kind) {
        pp = &b->next;
        continue;
      }
      *pp = b->next;
      if (kind == OBJ_LIVE) amod_live_close((amod_live *)b->p);
      else amod_asm_close((amod_assembler *)b->p);
      free(b);
    }
  }
}
static obj_box *obj_find(napi_env env, napi_value h, int32_t kind) {
  int64_t id = 0;
  if (napi_get_value_int64(env, h, &id) != napi_ok) return NULL;
  for (obj_box *b = g_objs; b; b = b->next)
    if (b->id == id && b->kind == kind && !b->close_pending) return b;
  return NULL;
}
static napi_value obj_new(napi_env env, int32_t kind, void *p, obj_box *dep) {
  napi_value out;
  obj_box *b = (obj_box *)calloc(1, sizeof *b);
  if (!b) return throw_msg(env, "out of memory");
  if (napi_create_int64(env, g_obj_next, &out) != napi_ok) {
    free(b);
    return throw_msg(env, "handle");
  }
  static int hooked = 0;
  if (!hooked) {
    napi_add_env_cleanup_hook(env, obj_cleanup, NULL);
    hooked = 1;
  }
  b->kind = kind;
  b->p = p;
  b->dep = dep;
  if (dep) ++dep->users;
  b->id = g_obj_next++;
  b->next = g_objs;
  g_objs = b;
  return out;
}

static obj_box *get_asm_box(napi_env env, napi_value v) {
  obj_box *b = obj_find(env, v, OBJ_ASM);
  if (!b) napi_throw_type_error(env, NULL, "expected an open assembler handle");
  return b;
}
static amod_assembler *get_asm(napi_env env, napi_value v) {
  obj_box *b = get_asm_box(env, v);
  return b ? (amod_assembler *)b->p : NULL;
}

/* asmClose(h) / liveClose(h): released now (an assembler: once its receivers close); a
   second close is a no-op */
static napi_value js_obj_close(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  void *data = NULL;
  size_t argc = 1;
  if (napi_get_cb_info(env, info, &argc, argv, NULL, &data) != napi_ok || argc < 1)
    return napi_throw_type_error(env, NULL, "close(handle)"), NULL;
  obj_box *b = obj_find(env, argv[0], (int32_t)(intptr_t)data);
  if (b) obj_release(b);
  return NULL;
}

static napi_value make_i32(napi_env env, int32_t v) {
  napi_value out;
  NAPI_TRY(env, napi_create_int32(env, v, &out));
  return out;
}

/* asmOpen(dir | null) -> handle (asmClose(handle), or closed at exit) */
static napi_value js_asm_open(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  char dir[4096] = {0};
  if (!is_nullish(env, argv[0])) {
    size_t n;
    if (napi_get_value_string_utf8(env, argv[0], dir, sizeof dir, &n) != napi_ok) return throw_msg(env, "bad dir");
  }
  amod_assembler *a;
  if (amod_asm_open(dir[0] ? dir : NULL, &a) != AMOD_SUCCESS) return throw_msg(env, "assembler");
  napi_value out = obj_new(env, OBJ_ASM, a, NULL);
  if (!out) amod_asm_close(a);
  return out;
}

/* asmMetadata(h, totalChunks, totalFileSize, chunkSize, nameBytes) -> status */
static napi_value js_asm_metadata(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  if (!get_args(env, info, 5, argv)) return NULL;
  amod_assembler *a = get_asm(env, argv[0]);
  if (!a) return NULL;
  int32_t tc, ts, cs;
  const uint8_t *nm;
  int32_t nn;
  if (napi_get_value_int32(env, argv[1], &tc) != napi_ok || napi_get_value_int32(env, argv[2], &ts) != napi_ok ||
      napi_get_value_int32(env, argv[3], &cs) != napi_ok || !get_u8(env, argv[4], &nm, &nn))
    return NULL;
  return make_i32(env, amod_asm_metadata(a, tc, ts, cs, nm, nn));
}

/* asmChunk(h, seq, data, crcValid) -> 1 stored / 0 ignored */
static napi_value js_asm_chunk(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return NULL;
  amod_assembler *a = get_asm(env, argv[0]);
  if (!a) return NULL;
  int32_t seq;
  bool crc;
  const uint8_t *d;
  int32_t n;
  if (napi_get_value_int32(env, argv[1], &seq) != napi_ok || !get_u8(env, argv[2], &d, &n) ||
      napi_get_value_bool(env, argv[3], &crc) != napi_ok)
    return NULL;
  return make_i32(env, amod_asm_chunk(a, seq, d, n, crc ? 1 : 0));
}

static napi_value bytes_from(napi_env env, const uint8_t *p, int64_t n) {
  napi_value ab, ta;
  void *q;
  NAPI_TRY(env, napi_create_arraybuffer(env, (size_t)(n > 0 ? n : 0), &q, &ab));
  if (n > 0) memcpy(q, p, (size_t)n);
  NAPI_TRY(env, napi_create_typedarray(env, napi_uint8_array, (size_t)(n > 0 ? n : 0), ab, 0, &ta));
  return ta;
}

/* asmState(h) -> {totalChunks, totalFileSize, chunkSize, receivedCount, crcErrors, complete,
   framesDecoded, frameErrors, bitmap: Uint8Array | null, fileName: Uint8Array} */
static napi_value js_asm_state(napi_env env, napi_callback_info info) {
  napi_value argv[1], out, v;
  if (!get_args(env, info, 1, argv)) return NULL;
  amod_assembler *a = get_asm(env, argv[0]);
  if (!a) return NULL;
  amod_asm_info st;
  amod_asm_state(a, &st);
  NAPI_TRY(env, napi_create_object(env, &out));
  const struct { const char *k; int32_t v; } f[] = {
      {"totalChunks", st.total_chunks}, {"totalFileSize", st.total_size}, {"chunkSize", st.chunk_size},
      {"receivedCount", st.received}, {"crcErrors", st.crc_errors}, {"framesDecoded", st.frames_decoded},
      {"frameErrors", st.frame_errors}};
  for (size_t i = 0; i < sizeof f / sizeof f[0]; ++i) {
    NAPI_TRY(env, napi_create_int32(env, f[i].v, &v));
    NAPI_TRY(env, napi_set_named_property(env, out, f[i].k, v));
  }
  NAPI_TRY(env, napi_get_boolean(env, st.complete != 0, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "complete", v));
  if (st.has_bitmap) {
    const int64_t n = amod_asm_bitmap(a, NULL, 0);
    uint8_t *b = (uint8_t *)malloc((size_t)(n > 0 ? n : 1));
    amod_asm_bitmap(a, b, n);
    v = bytes_from(env, b, n);
    free(b);
    if (!v) return NULL;
  } else {
    NAPI_TRY(env, napi_get_null(env, &v));
  }
  NAPI_TRY(env, napi_set_named_property(env, out, "bitmap", v));
  const int64_t nn = amod_asm_name(a, NULL, 0);
  uint8_t *nm = (uint8_t *)malloc((size_t)(nn > 0 ? nn : 1));
  amod_asm_name(a, nm, nn);
  v = bytes_from(env, nm, nn);
  free(nm);
  if (!v) return NULL;
  NAPI_TRY(env, napi_set_named_property(env, out, "fileName", v));
  return out;
}

/* asmMissing(h) -> Int32Array */
static napi_value js_asm_missing(napi_env env, napi_callback_info info) {
  napi_value argv[1], ab, ta;
  if (!get_args(env, info, 1, argv)) return NULL;
  amod_assembler *a = get_asm(env, argv[0]);
  if (!a) return NULL;
  const int64_t n = amod_asm_missing(a, NULL, 0);
  void *p;
  NAPI_TRY(env, napi_create_arraybuffer(env, (size_t)n * 4, &p, &ab));
  amod_asm_missing(a, (int32_t *)p, n);
  NAPI_TRY(env, napi_create_typedarray(env, napi_int32_array, (size_t)n, ab, 0, &ta));
  return ta;
}

/* asmFile(h) -> Uint8Array, or a negative status (RangeError / TypeError in JS) */
static napi_value js_asm_file(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  amod_assembler *a = get_asm(env, argv[0]);
  if (!a) return NULL;
  const int64_t n = amod_asm_file(a, NULL, 0);
  if (n < 0) return make_i32(env, (int32_t)n);
  napi_value ab, ta;
  void *p;
  NAPI_TRY(env, napi_create_arraybuffer(env, (size_t)n, &p, &ab));
  const int64_t m = amod_asm_file(a, (uint8_t *)p, n);
  if (m < 0) return make_i32(env, (int32_t)m);
  NAPI_TRY(env, napi_create_typedarray(env, napi_uint8_array, (size_t)n, ab, 0, &ta));
  return ta;
}

/* receiveStream(samples, cfg, asmHandle, device) -> {frames: ArrayBuffer of amod_stream_frame,
   nframes, refineFail: Float64Array, framesDecoded, frameErrors} */
static napi_value js_receive_stream(napi_env env, napi_callback_info info) {
  napi_value argv[4], out, v, ab;
  if (!get_args(env, info, 4, argv)) return NULL;
  float *x;
  size_t n;
  if (!typed(env, argv[0], napi_float32_array, (void **)&x, &n)) return throw_msg(env, "expected a Float32Array");
  amod_cfg c;
  if (!to_cfg(env, argv[1], &c)) return NULL;
  amod_assembler *a = get_asm(env, argv[2]);
  if (!a) return NULL;
  int32_t dev = 0;
  napi_get_value_int32(env, argv[3], &dev);
  amod_ctx *ctx = get_ctx(env, dev);
  if (!ctx) return NULL;
  const int64_t cap = (int64_t)(n / 4096) + 64;
  amod_stream_frame *fr = (amod_stream_frame *)calloc((size_t)cap, sizeof(amod_stream_frame));
  int64_t *rf = (int64_t *)calloc(4096, sizeof(int64_t));
  int64_t nf = 0;
  amod_stream_stats st;
  const int rc = amod_stream_receive(ctx, &c, x, (int64_t)n, a, fr, cap, &nf, rf, 4096, &st);
  if (rc != AMOD_SUCCESS) {
    free(fr); free(rf);
    return throw_msg(env, amod_last_error(ctx));
  }
  const int64_t k = nf < cap ? nf : cap;
  void *p;
  NAPI_TRY(env, napi_create_object(env, &out));
  NAPI_TRY(env, napi_create_arraybuffer(env, (size_t)k * sizeof(amod_stream_frame), &p, &ab));
  memcpy(p, fr, (size_t)k * sizeof(amod_stream_frame));
  NAPI_TRY(env, napi_set_named_property(env, out, "frames", ab));
  NAPI_TRY(env, napi_create_int64(env, k, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "nframes", v));
  const int64_t nr = st.nrefine_fail < 4096 ? st.nrefine_fail : 4096;
  NAPI_TRY(env, napi_create_arraybuffer(env, (size_t)nr * 8, &p, &ab));
  for (int64_t i = 0; i < nr; ++i) ((double *)p)[i] = (double)rf[i];
  NAPI_TRY(env, napi_create_typedarray(env, napi_float64_array, (size_t)nr, ab, 0, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "refineFail", v));
  NAPI_TRY(env, napi_create_int64(env, st.frames_decoded, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "framesDecoded", v));
  NAPI_TRY(env, napi_create_int64(env, st.frame_errors, &v));
  NAPI_TRY(env, napi_set_named_property(env, out, "frameErrors", v));
  free(fr);
  free(rf);
  return out;
}

/* ------------------------------------------------- live receiver (processAudioBlock) */
static amod_live *get_live(napi_env env, napi_value v) {
  obj_box *b = obj_find(env, v, OBJ_LIVE);
  if (!b) {
    napi_throw_type_error(env, NULL, "expected an open live receiver handle");
    return NULL;
  }
  return (amod_live *)b->p;
}

/* liveOpen(cfg, assemblerHandle, device) -> handle (liveClose(handle), or closed at exit) */
static napi_value js_live_open(napi_env env, napi_callback_info info) {
  napi_value argv[3], out;
  if (!get_args(env, info, 3, argv)) return NULL;
  amod_cfg c;
  if (!to_cfg(env, argv[0], &c)) return NULL;
  obj_box *ab = get_asm_box(env, argv[1]);
  if (!ab) return NULL;
  int32_t dev = 0;
  napi_get_value_int32(env, argv[2], &dev);
  amod_ctx *ctx = get_ctx(env, dev);
  if (!ctx) return NULL;
  amod_live *lv;
  if (amod_live_open(ctx, &c, (amod_assembler *)ab->p, &lv) != AMOD_SUCCESS) return throw_msg(env, amod_last_error(ctx));
  out = obj_new(env, OBJ_LIVE, lv, ab);
  if (!out) amod_live_close(lv);
  return out;
}

/* liveProcess(handle, Float32Array) -> ArrayBuffer (one amod_stream_frame) | null */
static napi_value js_live_process(napi_env env, napi_callback_info info) {
  napi_value argv[2], out;
  if (!get_args(env, info, 2, argv)) return NULL;
  amod_live *lv = get_live(env, argv[0]);
  if (!lv) return NULL;
  float *x;
  size_t n;
  if (!typed(env, argv[1], napi_float32_array, (void **)&x, &n)) return throw_msg(env, "expected a Float32Array");
  amod_stream_frame f;
  int32_t has = 0;
  if (amod_live_process_block(lv, x, (int64_t)n, &f, &has) != AMOD_SUCCESS) return throw_msg(env, amod_last_error(NULL));
  if (!has) {
    NAPI_TRY(env, napi_get_null(env, &out));
    return out;
  }
  void *p;
  NAPI_TRY(env, napi_create_arraybuffer(env, sizeof f, &p, &out));
  memcpy(p, &f, sizeof f);
  return out;
}

/* liveState(handle) -> {state, acScanPos, preambleGlobalPos, expectedFrameEnd, metaReceived,
   chunkSize, totalWritten, framesDecoded, frameErrors, refineFails} */
static napi_value js_live_state(napi_env env, napi_callback_info info) {
  napi_value argv[1], out, v;
  if (!get_args(env, info, 1, argv)) return NULL;
  amod_live *lv = get_live(env, argv[0]);
  if (!lv) return NULL;
  amod_stream_state st;
  amod_live_stats ls;
  amod_live_state(lv, &st, &ls);
  NAPI_TRY(env, napi_create_object(env, &out));
#define SETNUM(name, val)                                                               \
  do {                                                                                  \
    NAPI_TRY(env, napi_create_double(env, (double)(val), &v));                          \
    NAPI_TRY(env, napi_set_named_property(env, out, name, v));                          \
  } while (0)
  SETNUM("state", st.state);
  SETNUM("acScanPos", st.ac_pos);
  SETNUM("preambleGlobalPos", st.pre_pos);
  SETNUM("expectedFrameEnd", st.frame_end);
  SETNUM("metaReceived", st.meta_received);
  SETNUM("chunkSize", st.chunk_size);
  SETNUM("totalWritten", ls.total_written);
  SETNUM("framesDecoded", ls.frames_decoded);
  SETNUM("frameErrors", ls.frame_errors);
  SETNUM("refineFails", ls.refine_fails);
#undef SETNUM
  return out;
}

/* diagnostics (AMODEM_SEGV_TRACE=1): a crash prints the native stack (library + offset per
   frame, for addr2line) before the default action */
static void segv_trace(int sig) {
  void *fr[64];
  const int n = backtrace(fr, 64);
  static const char msg[] = "[amodem.node] fatal signal, native stack:\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static napi_value init(napi_env env, napi_value exports) {
  if (getenv("AMODEM_SEGV_TRACE")) {
    signal(SIGSEGV, segv_trace);
    signal(SIGBUS, segv_trace);
  }
  const napi_property_descriptor props[] = {
      {"decode", NULL, js_decode, NULL, NULL, NULL, napi_enumerable, NULL},
      {"decodeAsync", NULL, js_decode_async, NULL, NULL, NULL, napi_enumerable, NULL},
      {"residentUpload", NULL, js_resident_upload, NULL, NULL, NULL, napi_enumerable, NULL},
      {"residentDecodeAsync", NULL, js_resident_decode_async, NULL, NULL, NULL, napi_enumerable, NULL},
      {"residentFree", NULL, js_resident_free, NULL, NULL, NULL, napi_enumerable, NULL},
      {"loopback", NULL, js_loopback, NULL, NULL, NULL, napi_enumerable, NULL},
      {"crc32", NULL, js_crc32, NULL, NULL, NULL, napi_enumerable, NULL},
      {"preamble1", NULL, js_preamble1, NULL, NULL, NULL, napi_enumerable, NULL},
      {"txLegacy", NULL, js_tx_legacy, NULL, NULL, NULL, napi_enumerable, NULL},
      {"txMeta", NULL, js_tx_meta, NULL, NULL, NULL, napi_enumerable, NULL},
      {"txChunk", NULL, js_tx_chunk, NULL, NULL, NULL, napi_enumerable, NULL},
      {"txTestSignal", NULL, js_tx_test, NULL, NULL, NULL, napi_enumerable, NULL},
      {"estimateFrameSamples", NULL, js_estimate, NULL, NULL, NULL, napi_enumerable, NULL},
      {"numDataSubs", NULL, js_num_data_subs, NULL, NULL, NULL, napi_enumerable, NULL},
      {"payloadStride", NULL, js_payload_stride, NULL, NULL, NULL, napi_enumerable, NULL},
      {"abiVersion", NULL, js_abi, NULL, NULL, NULL, napi_enumerable, NULL},
      {"asmOpen", NULL, js_asm_open, NULL, NULL, NULL, napi_enumerable, NULL},
      {"asmMetadata", NULL, js_asm_metadata, NULL, NULL, NULL, napi_enumerable, NULL},
      {"asmChunk", NULL, js_asm_chunk, NULL, NULL, NULL, napi_enumerable, NULL},
      {"asmState", NULL, js_asm_state, NULL, NULL, NULL, napi_enumerable, NULL},
      {"asmMissing", NULL, js_asm_missing, NULL, NULL, NULL, napi_enumerable, NULL},
      {"asmFile", NULL, js_asm_file, NULL, NULL, NULL, napi_enumerable, NULL},
      {"asmClose", NULL, js_obj_close, NULL, NULL, NULL, napi_enumerable, (void *)(intptr_t)OBJ_ASM},
      {"receiveStream", NULL, js_receive_stream, NULL, NULL, NULL, napi_enumerable, NULL},
      {"liveOpen", NULL, js_live_open, NULL, NULL, NULL, napi_enumerable, NULL},
      {"liveProcess", NULL, js_live_process, NULL, NULL, NULL, napi_enumerable, NULL},
      {"liveState", NULL, js_live_state, NULL, NULL, NULL, napi_enumerable, NULL},
      {"liveClose", NULL, js_obj_close, NULL, NULL, NULL, napi_enumerable, (void *)(intptr_t)OBJ_LIVE},
  };
  if (napi_define_properties(env, exports, sizeof props / sizeof props[0], props) != napi_ok) return NULL;
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
