/*
 * amodem.h — C ABI of the MI355X-native OFDM demodulator (libamodem.so).
 *
 * Drop-in engine behind the receive half of playok/audio-modem's modem.js.
 * Plain C types only; no exceptions, no torch types. Every entry point returns
 * an int status (AMOD_SUCCESS or a negative AMOD_ERR_*); per-frame decode
 * outcomes are reported in amod_result.status using the reference's error set.
 *
 * Reference interfaces each entry point replaces (file:line in modem.js):
 *   amod_decode_*(mode = AMOD_MODE_RECEIVED) ... decodeReceivedSignal   modem.js:557-654
 *   amod_decode_*(mode = AMOD_MODE_CHUNK)    ... decodeChunkFrame       modem.js:770-803
 *   amod_config_preset                       ... OFDM_CONFIGS / setOFDMConfig modem.js:69-98
 *   amod_estimate_frame_samples              ... estimateFrameSamples   modem.js:863-874
 *   amod_crc32                               ... crc32                  modem.js:443-457
 *   amod_tx_legacy / amod_tx_meta / amod_tx_chunk / amod_tx_test_signal
 *                                            ... buildTransmitSignal 498-555, buildMetadataFrame 758,
 *                                                buildDataChunkFrame 763, generateTestSignal 914-973
 *   amod_preamble1                           ... generatePreambleSymbol1 modem.js:158-170
 * The reference's JS binds none of these today; INTEGRATION.md shows the N-API
 * binding (audio-modem_amd/csrc/napi_amodem.c) a maintainer adds.
 */
#ifndef AMODEM_H
#define AMODEM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMOD_ABI_VERSION 1
#define AMOD_MAX_PILOTS 32

/* ---- API status (return values) ---- */
#define AMOD_SUCCESS 0
#define AMOD_ERR_ARG (-1)     /* invalid argument / config                     */
#define AMOD_ERR_HIP (-2)     /* HIP runtime failure (see amod_last_error)     */
#define AMOD_ERR_NOMEM (-3)   /* device or host allocation failed              */
#define AMOD_ERR_NODEV (-4)   /* no usable gfx950 device                       */

/* ---- modulations (Constellations, modem.js:101-105) ---- */
#define AMOD_BPSK 0
#define AMOD_QPSK 1
#define AMOD_QAM16 2

/* ---- decode modes ---- */
#define AMOD_MODE_RECEIVED 0 /* decodeReceivedSignal: preprocess + detect + demod + parse */
#define AMOD_MODE_CHUNK 1    /* decodeChunkFrame: frame starts at preamble 1             */
#define AMOD_MODE_LOOPBACK 2 /* analyzeLoopback's receive core (exact kernel): detection
                                with the cross-correlation fallback, fine timing without the
                                0.1 cut-off, channel estimate and the raw decoded bytes      */

/* ---- decode option bits ---- */
#define AMOD_OPT_FORCE_EXACT 1u /* run every frame through the exact-replica kernel */
/* NOT reference behaviour, opt-in (BASELINE C5's noisy-channel path): with repetition > 1
   and BPSK / QPSK, each group of `rep` repeated bits is decided by the sign of its summed
   soft values (BPSK: the phase-corrected real part; QPSK: max-log per bit) instead of
   majorityVote's hard vote (modem.js:487-495). Such frames run on the exact kernel. */
#define AMOD_OPT_SOFT_COMBINE 2u

/* ---- per-frame status (the reference's error strings, modem.js) ---- */
#define AMOD_OK 0
#define AMOD_E_PREAMBLE 1        /* 'Preamble not detected'                     */
#define AMOD_E_LOW_CORR 2        /* 'Preamble not detected (low correlation)'   */
#define AMOD_E_SHORT_CE 3        /* 'Signal too short for CE'                   */
#define AMOD_E_NO_DATA 4         /* 'No data after CE'                          */
#define AMOD_E_DECODED_SHORT 5   /* 'Decoded data too short'                    */
#define AMOD_E_SHORT_HEADER 6    /* 'Decoded data too short for header'         */
#define AMOD_E_INVALID_LEN 7     /* `Invalid data length: ${aux}`               */
#define AMOD_E_META_SHORT 8      /* 'Metadata frame too short'                  */
#define AMOD_E_META_TRUNC 9      /* 'Metadata frame truncated'                  */
#define AMOD_E_CHUNK_SHORT 10    /* 'Data chunk frame too short'                */
#define AMOD_E_CHUNK_TRUNC 11    /* 'Data chunk truncated'                      */
#define AMOD_E_FRAME_SHORT_CE 12 /* 'Frame too short for CE'                    */
#define AMOD_E_UNKNOWN_TYPE 13   /* `Unknown frame type: 0x${aux.toString(16)}` */
#define AMOD_E_CAPACITY 100      /* not a reference outcome: the frame exceeds the workspace
                                    reserved by amod_reserve (device path); reserve more  */

/* ---- amod_result.flags: why a frame was (re)decoded by the exact kernel ---- */
#define AMOD_FLAG_FORCED (1 << 0)    /* AMOD_OPT_FORCE_EXACT                        */
#define AMOD_FLAG_NONFINITE (1 << 1) /* NaN/Inf samples                             */
#define AMOD_FLAG_BIG (1 << 2)       /* frame longer than the LDS-resident capacity */
#define AMOD_FLAG_COARSE (1 << 3)    /* Schmidl-Cox decision within guard band      */
#define AMOD_FLAG_FINE (1 << 4)      /* fine-timing argmax within guard band        */
#define AMOD_FLAG_CHANNEL (1 << 5)   /* |H|^2 near the 1e-10 threshold              */
#define AMOD_FLAG_PHASE (1 << 6)     /* pilot |eqRe| near the 1e-6 threshold        */
#define AMOD_FLAG_DEMAP (1 << 7)     /* a constellation decision within guard band  */
#define AMOD_FLAG_THRESH (1 << 8)    /* preprocess peak near the 1e-6 threshold     */
#define AMOD_FLAG_SPAN (1 << 9)      /* the parse reads bytes past the symbols the fast
                                        path demodulated (signal energy ended early)   */
#define AMOD_FLAG_SOFT (1 << 10)     /* AMOD_OPT_SOFT_COMBINE: demodulated by the exact
                                        kernel after the fast path's detection         */
#define AMOD_FLAG_REPLAY (1 << 11)   /* preambleIdx from the exact replica's detection
                                        (COARSE / FINE / THRESH), symbols demodulated
                                        by the fast path under its guards              */
#define AMOD_FLAG_EXACT (1 << 15)    /* result produced by the exact-replica kernel */

/* OFDM parameters + modulation; mirrors OFDM (modem.js:69-98) */
typedef struct amod_cfg {
  int32_t fft_size; /* must be 512 */
  int32_t cp_len;
  int32_t symbol_len; /* fft_size + cp_len */
  int32_t sample_rate;
  int32_t sub_start, sub_end; /* in-band subcarriers, inclusive; sub_end < fft_size/2 */
  int32_t npilots;
  int32_t pilots[AMOD_MAX_PILOTS];
  int32_t modulation; /* AMOD_BPSK / AMOD_QPSK / AMOD_QAM16 */
  int32_t repetition; /* >= 1 (majorityVote n) */
} amod_cfg;

/* One record per frame (96 bytes). Offsets index the frame's payload slot. */
typedef struct amod_result {
  int32_t status;       /* AMOD_OK or AMOD_E_*                                           */
  int32_t preamble_idx; /* startIdx (RECEIVED mode); -1 when the reference omits it      */
  int32_t coarse_idx;   /* Schmidl-Cox index (exact kernel: bit-exact; fast: in plateau) */
  int32_t frame_type;   /* 0 legacy, 0xFE meta, 0xFF data, other byte / -1 if none       */
  int32_t aux;          /* dataLen for AMOD_E_INVALID_LEN, type byte for UNKNOWN_TYPE    */
  int32_t nbytes;       /* decoded bytes (after vote) stored in the payload slot         */
  int32_t name_off, name_len;
  int32_t data_off, data_len;
  int32_t seq_num, total_chunks, total_size, chunk_size;
  uint32_t expected_crc, actual_crc;
  int32_t crc_valid;
  int32_t nbits;       /* demodulated bits before vote                                  */
  int32_t flags;       /* AMOD_FLAG_*                                                   */
  float fine_metric;   /* best normalised cross-correlation                             */
  int32_t payload_valid; /* leading payload-slot bytes that hold decoded bytes: all nbytes
                            (exact kernel), or the header..CRC prefix the parse reads (fast
                            kernel: symbols past the CRC are not demodulated). Bytes past it
                            are not written by the device path (zero from amod_decode_host) */
  int32_t reserved[3];
} amod_result;

typedef struct amod_ctx amod_ctx;

/* ---- lifecycle ---- */
int amod_open(int device, amod_ctx **out); /* binds a HIP device; own stream + workspace */
int amod_close(amod_ctx *ctx);
const char *amod_last_error(const amod_ctx *ctx); /* NULL ctx: last global error */
int amod_abi_version(void);

/* ---- configuration & sizing ---- */
/* name: 'standard' | 'acoustic' | 'narrowband' (unknown -> standard, modem.js:96) */
int amod_config_preset(const char *name, int32_t modulation, int32_t repetition, amod_cfg *out);
int32_t amod_num_data_subs(const amod_cfg *cfg);
int32_t amod_estimate_frame_samples(const amod_cfg *cfg, int32_t payload_bytes);
/* bytes each frame's payload slot needs for frames up to max_frame_len samples */
int64_t amod_payload_stride(const amod_cfg *cfg, int64_t max_frame_len);
/* pre-size the workspace so a later decode of this shape allocates nothing
   (required before capturing amod_decode_device into a hipGraph). max_frame_len also
   sets the device path's fast-path capacity from this call on (default 65536 samples):
   on amod_decode_device a frame's route (fast kernels or the exact replica, visible in
   amod_result.flags / coarse_idx / fine_metric / payload_valid; never in the reference's
   fields) depends on the frame, the options and the latest reservation only. Host
   decodes size their own capacity from their longest frame. After a decode was captured
   into a graph, a buffer that must grow is kept (not freed) until amod_close, so the
   graph's replays stay valid. */
int amod_reserve(amod_ctx *ctx, const amod_cfg *cfg, int32_t nframes, int64_t max_frame_len);

/* ---- decode ----
 * Frames are slices [offsets[i], offsets[i]+lengths[i]) of one float32 sample
 * buffer (device path: the buffer must be 16-byte aligned). Results go to results[i]; decoded bytes to payload + i*payload_stride.
 * amod_decode_device: every pointer is device memory; enqueued on `stream`
 * (hipStream_t, NULL = the context's stream); returns without synchronising.
 * amod_decode_host: host pointers; copies over PCIe and synchronises.
 * debug (device, optional): per-frame amod_debug records for parity tests.   */
int amod_decode_device(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples,
                       const int64_t *offsets, const int32_t *lengths, int32_t nframes,
                       amod_result *results, uint8_t *payload, int64_t payload_stride, uint32_t options,
                       void *stream);
int amod_decode_host(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples,
                     int64_t nsamples, const int64_t *offsets, const int32_t *lengths, int32_t nframes,
                     amod_result *results, uint8_t *payload, int64_t payload_stride, uint32_t options);
/* amod_decode_host with progress reports (additive; the Node binding formats decodeBatch's
 * result objects while later frames decode): progress(user, done) runs on a helper thread
 * of the call (one at a time, done increasing) whenever records and payload slots
 * [0, done) are in the caller's buffers; its last call has done = nframes, and every call
 * has returned before amod_decode_host_progress does (no call for an empty batch). The
 * calling thread meanwhile keeps uploading the next pieces. A frame's
 * outputs reach the caller as soon as its uploaded piece (64 MB of samples) is decoded. */
typedef void (*amod_progress_fn)(void *user, int32_t frames_done);
int amod_decode_host_progress(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples,
                              int64_t nsamples, const int64_t *offsets, const int32_t *lengths,
                              int32_t nframes, amod_result *results, uint8_t *payload,
                              int64_t payload_stride, uint32_t options, amod_progress_fn progress,
                              void *user);
int amod_synchronize(amod_ctx *ctx);

/* ---- a depth-2 pipeline of device decodes (additive; no reference counterpart) ----
 * Consecutive batches alternate between two caller-owned contexts of one device, each
 * decoding on one of the pipe's two streams, so batch i + 1's detection overlaps batch i's
 * demodulation. Fastest use (stream = NULL or the slot's stream): enqueue each batch's
 * inputs on amod_pipe_next_stream(p) (hipStream_t), decode, and read its results on that
 * same stream: plain stream order. With another `stream`, a decode starts once that
 * stream reaches the call, and decode i's results are ordered on it when decode i + 1 has
 * been enqueued (whatever stream that call passes: the join goes to the stream that issued
 * decode i), or after amod_pipe_flush(stream) (two cross-queue signals per batch: less
 * overlap). amod_pipe_synchronize waits on the host. One host thread per pipe; the
 * contexts must take no other work while it runs, and a context closed before the pipe
 * must have its pipe decodes finished first (amod_pipe_synchronize / amod_pipe_close;
 * the Python Demodulator closes its pipes itself). */
typedef struct amod_pipe amod_pipe;
int amod_pipe_open(amod_ctx *a, amod_ctx *b, amod_pipe **out);
int amod_pipe_close(amod_pipe *p); /* waits for its decodes and destroys its two streams;
                                      the contexts stay open */
void *amod_pipe_next_stream(const amod_pipe *p);
int amod_pipe_decode_device(amod_pipe *p, const amod_cfg *cfg, int32_t mode, const float *samples,
                            const int64_t *offsets, const int32_t *lengths, int32_t nframes,
                            amod_result *results, uint8_t *payload, int64_t payload_stride,
                            uint32_t options, void *stream);
int amod_pipe_flush(amod_pipe *p, void *stream);
int amod_pipe_synchronize(amod_pipe *p);

/* kernel timing: when enabled, every decode brackets each launch of the fast path
   (k_detect, k_demod) and k_decode_exact with hipEvents on the launch
   stream; amod_kernel_times waits for them, returns the accumulated milliseconds of
   the fast path and of the exact kernel and the decode count, and resets */
int amod_set_profiling(amod_ctx *ctx, int enable);
int amod_kernel_times(amod_ctx *ctx, double *fast_ms, int64_t *fast_launches, double *exact_ms,
                      int64_t *exact_launches);
/* the same events split by launch: ms[0..2] = k_detect (k_chunk_prep in chunk mode),
   k_demod up to the launch stream's join with the second stream (so it includes any
   part of list A's exact chain that outlasts k_demod), list B's k_decode_exact;
   accumulated over *n decodes; resets like amod_kernel_times */
int amod_kernel_breakdown(amod_ctx *ctx, double *ms, int64_t *n);
/* the stage slots of amod_kernel_stages (ms[AMOD_STAGE_*], milliseconds summed over *n
   launch sequences; resets like amod_kernel_times). A device decode is one launch
   sequence; amod_decode_host launches one per uploaded piece (64 MB) whose frames have
   landed, so there *n counts pieces, not host calls. */
enum {
  AMOD_STAGE_DETECT = 0,     /* k_detect / k_chunk_prep */
  AMOD_STAGE_DEMOD = 1,      /* k_demod alone (launch stream) */
  AMOD_STAGE_EXACT_B = 2,    /* list B's k_decode_exact (frames k_demod listed) */
  AMOD_STAGE_AUX = 3,        /* second stream: list A's k_decode_exact + the replay k_demod,
                                from the end of k_detect (runs beside k_demod) */
  AMOD_STAGE_JOIN_WAIT = 4,  /* end of k_demod -> the launch stream joined the second one */
  AMOD_STAGE_DEMOD_PATH = 5, /* k_demod + the join wait (amod_kernel_breakdown's ms[1]) */
  AMOD_STAGE_COUNT = 6
};
int amod_kernel_stages(amod_ctx *ctx, double *ms, int32_t nslots, int64_t *n);
/* whether list A's exact chain ran beside k_demod (profiled decodes only, collected by
   amod_kernel_stages): of the decodes since the last call, *listed had a frame on list A
   (detection listed it), *beside started that frame's replica before k_demod's last wave
   ended, and *lead_us sums k_demod's end minus the replica's start (device real-time
   clock, microseconds; positive = beside). Resets. Not a reference function: the
   scheduling evidence for the second stream. */
int amod_aux_overlap(amod_ctx *ctx, int64_t *listed, int64_t *beside, double *lead_us);

/* parity-test view of one frame's intermediates (filled when debug != NULL) */
#define AMOD_DBG_BAND 256
#define AMOD_DBG_SYMS 256
typedef struct amod_debug {
  double mean, mx;             /* preprocess                                    */
  double coarse_metric;        /* best Schmidl-Cox metric                       */
  int32_t coarse_lo, coarse_hi; /* candidate plateau [lo, hi]                   */
  double fine_metric;
  int32_t fine_idx, nsym;
  double h_re[AMOD_DBG_BAND], h_im[AMOD_DBG_BAND];   /* channel estimate, band order */
  double x_re[AMOD_DBG_BAND], x_im[AMOD_DBG_BAND];   /* FFT of data symbol 0 (band)  */
  double eq_re[AMOD_DBG_BAND], eq_im[AMOD_DBG_BAND]; /* equalised symbol 0 (band)    */
  double phase[AMOD_DBG_SYMS];                       /* pilot phase per data symbol  */
} amod_debug;
int amod_decode_device_debug(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples,
                             const int64_t *offsets, const int32_t *lengths, int32_t nframes,
                             amod_result *results, uint8_t *payload, int64_t payload_stride,
                             uint32_t options, void *stream, amod_debug *debug);

/* analyzeLoopback (modem.js:975-1082) receive core for one host signal: fills
   res (status AMOD_E_PREAMBLE = not detected even by the cross-correlation fallback
   (modem.js:235-284), AMOD_E_SHORT_CE = no room for the CE symbol; preamble_idx =
   startIdx; nbytes = decoded bytes after the vote, stored in bytes[0, min(nbytes, cap))),
   dbg->fine_metric (bestMetric, -inf if no offset passed the gate) and dbg->h_re/h_im
   (the channel estimate over the band). The caller finishes the report (channel
   magnitude, pilot SNR, BER, quality) with the reference's own arithmetic.        */
int amod_analyze_loopback(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t nsamples,
                          amod_result *res, amod_debug *dbg, uint8_t *bytes, int64_t cap);

/* diagnostics: with AMOD_STAMPS set in the environment, the fast kernel records
   32 s_memtime marks per frame (wave 0); copies up to cap of them, returns count */
int64_t amod_debug_stamps(amod_ctx *ctx, uint64_t *out, int64_t cap);

/* ---- host utilities (reference-equivalent, bit-exact) ---- */
uint32_t amod_crc32(const uint8_t *data, size_t n);
int amod_preamble1(const amod_cfg *cfg, float *out); /* symbol_len floats */
/* transmit builders for synthetic input; return sample count, out may be NULL to size */
int64_t amod_tx_legacy(const amod_cfg *cfg, const uint8_t *data, int32_t len, const uint8_t *name,
                       int32_t name_len, float *out);
int64_t amod_tx_meta(const amod_cfg *cfg, int32_t total_chunks, int32_t total_size, int32_t chunk_size,
                     const uint8_t *name, int32_t name_len, float *out);
int64_t amod_tx_chunk(const amod_cfg *cfg, const uint8_t *data, int32_t len, int32_t seq, float *out);
int64_t amod_tx_test_signal(const amod_cfg *cfg, float *out);
/* ---- GPU transmitter (k_tx): modulateOFDM (modem.js:322-362) + buildTransmitSignal (498-555) /
 * buildChunkOFDMFrame (718-756), bit-exact with the builders above.
 * Packets are the bytes the reference frames: buildTransmitSignal's packet (amod_packet_legacy),
 * buildMetadataPayload (amod_packet_meta, modem.js:666-692) or buildDataChunkPayload
 * (amod_packet_chunk, 694-714); each returns its size (out NULL: sizing only).
 * amod_tx_silence gives the builder's silence lengths; amod_tx_frame_samples the
 * frame length. amod_tx_device: every pointer device memory; frame f's packet is
 * packets[pkt_off[f], +pkt_len[f]), its samples go to out + out_off[f]; enqueued on
 * `stream` (NULL = the context's stream). */
#define AMOD_TX_LEGACY 0 /* buildTransmitSignal: 0.3 / 0.2 s silence (acoustic 0.5 / 0.5) */
#define AMOD_TX_META 1   /* buildMetadataFrame (first frame): 0.3 s (acoustic 0.5) / 0.02 s */
#define AMOD_TX_CHUNK 2  /* buildDataChunkFrame: 0.05 s / 0.02 s */
int64_t amod_packet_legacy(const uint8_t *data, int32_t len, const uint8_t *name, int32_t name_len, uint8_t *out);
int64_t amod_packet_meta(int32_t total_chunks, int32_t total_size, int32_t chunk_size, const uint8_t *name,
                         int32_t name_len, uint8_t *out);
int64_t amod_packet_chunk(const uint8_t *data, int32_t len, int32_t seq, uint8_t *out);
int amod_tx_silence(const amod_cfg *cfg, int32_t kind, int32_t *pre, int32_t *post);
int64_t amod_tx_frame_samples(const amod_cfg *cfg, int64_t pkt_len, int32_t pre, int32_t post);
int amod_tx_device(amod_ctx *ctx, const amod_cfg *cfg, const uint8_t *packets, const int64_t *pkt_off,
                   const int32_t *pkt_len, const int32_t *pre, const int32_t *post, int32_t nframes, float *out,
                   const int64_t *out_off, void *stream);
/* host staging of amod_tx_device: frames back to back in out (out_off filled, may be
   NULL); returns the total sample count (out NULL: sizing only), < 0 on error */
int64_t amod_tx_host(amod_ctx *ctx, const amod_cfg *cfg, const uint8_t *packets, int64_t nbytes,
                     const int64_t *pkt_off, const int32_t *pkt_len, const int32_t *pre, const int32_t *post,
                     int32_t nframes, float *out, int64_t *out_off);
/* the synthetic legacy workload's packets (payload seed 0x9E3779B9 ^ (first+i)), back to back */
int64_t amod_synth_legacy_packets(int32_t nframes, int32_t first, int32_t payload_len, const uint8_t *name,
                                  int32_t name_len, uint8_t *out, int64_t *offsets, int32_t *lengths);
/* ---- chunk assembly (host): app.js ChunkAssembler (597-704) and the result dispatch of
 * StreamingReceiver._demodulateFrame (926-961), with the reference's quirks (assembler.cpp).
 * dir != NULL keeps chunks as files under dir (the IndexedDB store's stand-in), else memory.
 * amod_asm_chunk returns 1 if stored, 0 if ignored; amod_asm_file returns the file size
 * (out NULL: sizing) or one of the errors the reference throws: */
#define AMOD_ASM_RANGE_ERROR (-10) /* RangeError: negative sizes, a chunk past the file end */
#define AMOD_ASM_TYPE_ERROR (-11)  /* TypeError: assembleFile before any metadata frame     */
typedef struct amod_assembler amod_assembler;
typedef struct amod_asm_info {
  int32_t total_chunks, total_size, chunk_size; /* last metadata frame                     */
  int32_t received, crc_errors, complete;       /* receivedCount, crcErrors, isComplete()  */
  int32_t has_bitmap;                           /* a metadata frame created the bitmap     */
  int32_t frames_decoded, frame_errors;         /* StreamingReceiver counters (feed only)  */
  int32_t name_len, reserved;
  int64_t bitmap_len;                           /* -1 without bitmap                       */
} amod_asm_info;
int amod_asm_open(const char *dir, amod_assembler **out);
int amod_asm_close(amod_assembler *a);
int amod_asm_metadata(amod_assembler *a, int32_t total_chunks, int32_t total_size, int32_t chunk_size,
                      const uint8_t *name, int32_t name_len);
int amod_asm_chunk(amod_assembler *a, int32_t seq, const uint8_t *data, int32_t len, int32_t crc_valid);
int amod_asm_feed(amod_assembler *a, const amod_result *res, const uint8_t *payload, int64_t stride, int32_t n);
int amod_asm_state(const amod_assembler *a, amod_asm_info *out);
int64_t amod_asm_bitmap(const amod_assembler *a, uint8_t *out, int64_t cap);
int64_t amod_asm_name(const amod_assembler *a, uint8_t *out, int64_t cap);
int64_t amod_asm_missing(const amod_assembler *a, int32_t *out, int64_t cap);
int64_t amod_asm_file(const amod_assembler *a, uint8_t *out, int64_t cap);

/* ---- several GPUs from one host process ----
 * A group holds one context per listed device (a device may repeat). amod_group_decode_host
 * decodes a batch like amod_decode_host, cut into contiguous frame ranges of about equal
 * sample counts, one per device, all devices at once; every range's results and payload
 * rows land in the caller's arrays at their frame index (per-device D2H, no gather step).
 * frames_per_device (optional, group-size entries): the split used. */
typedef struct amod_group amod_group;
int amod_group_open(const int32_t *devices, int32_t ndev, amod_group **out);
int amod_group_close(amod_group *g);
int32_t amod_group_size(const amod_group *g);
amod_ctx *amod_group_context(amod_group *g, int32_t i);
int amod_group_decode_host(amod_group *g, const amod_cfg *cfg, int32_t mode, const float *samples, int64_t nsamples,
                           const int64_t *offsets, const int32_t *lengths, int32_t nframes, amod_result *results,
                           uint8_t *payload, int64_t payload_stride, uint32_t options, int32_t *frames_per_device);

/* Device-resident shards, one per group member (frames independent: modem.js:557,770, so
 * no exchange between devices). Shard k's pointers are memory on member k's device (as
 * amod_decode_device: samples 16-byte aligned, frames [offsets[i], offsets[i]+lengths[i])
 * of its own buffer); stream = a hipStream_t of that device, NULL = the member context's
 * stream. Every member's decode is enqueued from the calling thread and the call returns
 * without synchronising (amod_group_synchronize waits for the members' own streams).
 * Shards with nframes == 0 are skipped. */
typedef struct amod_shard {
  const float *samples;
  const int64_t *offsets;
  const int32_t *lengths;
  amod_result *results;
  uint8_t *payload;
  int64_t payload_stride;
  void *stream;
  int32_t nframes;
  int32_t reserved;
} amod_shard;
int amod_group_decode_device(amod_group *g, const amod_cfg *cfg, int32_t mode, const amod_shard *shards,
                             uint32_t options);
int amod_group_synchronize(amod_group *g);

/* A host batch made resident across a group once (the split of amod_group_decode_host:
 * contiguous frame ranges of about equal sample counts) and decoded from HBM as often as
 * the caller likes: amod_resident_decode runs amod_group_decode_device over the resident
 * shards and copies every member's records and payload rows into the caller's host arrays
 * at their frame index (one D2H per member, no gather), then synchronises. */
typedef struct amod_resident amod_resident;
int amod_group_upload(amod_group *g, const amod_cfg *cfg, const float *samples, int64_t nsamples,
                      const int64_t *offsets, const int32_t *lengths, int32_t nframes, amod_resident **out);
int amod_resident_decode(amod_resident *r, const amod_cfg *cfg, int32_t mode, uint32_t options,
                         amod_result *results, uint8_t *payload, int64_t payload_stride);
int32_t amod_resident_frames(const amod_resident *r, int32_t *frames_per_device);
int amod_resident_free(amod_resident *r);

/* ---- streaming receive: app.js StreamingReceiver (706-998) over a recorded stream ----
 * The stream is cut into 4096-sample blocks (the ScriptProcessor size; a last partial
 * block is completed with zeros) and run through the reference's receiver: EMA DC
 * removal, Schmidl-Cox scan, cross-correlation refine, frame collection, per-window
 * peak normalisation, decodeChunkFrame (GPU, chunk mode) and the ChunkAssembler
 * dispatch into `assembler` (NULL: a private one). frames[0..min(*nframes, max_frames))
 * receive every demodulated window: pos = preambleGlobalPos, end = expectedFrameEnd,
 * result = decodeChunkFrame's outcome (AMOD_E_STREAM_LOST: the window had left the
 * ring buffer, counted as a frame error). refine_fail lists preamble positions whose
 * refinement found no correlation >= 0.1 (app.js:880-884). samples: host memory.    */
#define AMOD_E_STREAM_LOST 101 /* not a decode outcome: getRange() returned null */
typedef struct amod_stream_frame {
  int64_t pos, end;
  int32_t window_len, reserved;
  amod_result result;
} amod_stream_frame;
typedef struct amod_stream_stats {
  int64_t nframes, nrefine_fail, frames_decoded, frame_errors; /* receiver counters */
  int64_t final_state, final_scan_pos;        /* RECV_STATE and acScanPos after the last block */
  int64_t ema_chunks_fixed;                    /* EMA chunks recomputed after the warm-up check */
  int64_t fine_host_positions;                 /* refine positions outside the GPU precompute */
  double t_ema_ms, t_fine_ms, t_decode_ms, t_host_ms, t_total_ms;
} amod_stream_stats;
/* processAudioBlock's DC removal (app.js:751-755) over a device buffer x[0, n) from a zero
 * EMA state: y (device) = f32(x - m) bit-exact, *end_state = the EMA state after x[n - 1],
 * *chunks_fixed = EMA chunks whose parallel warm-up had to be recomputed (diagnostics).
 * Either pointer may be NULL. stream 0: the context's stream; returns after it is done. */
int amod_dc_remove_device(amod_ctx *ctx, const float *x, int64_t n, float *y, double *end_state,
                          int64_t *chunks_fixed, void *stream);

int amod_stream_receive(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t n,
                        amod_assembler *assembler, amod_stream_frame *frames, int64_t max_frames,
                        int64_t *nframes, int64_t *refine_fail, int64_t max_refine_fail, amod_stream_stats *stats);

/* amod_stream_receive with the samples already in device memory (samples: a device
 * pointer to n floats; the stream is not copied). */
int amod_stream_receive_device(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t n,
                               amod_assembler *assembler, amod_stream_frame *frames, int64_t max_frames,
                               int64_t *nframes, int64_t *refine_fail, int64_t max_refine_fail,
                               amod_stream_stats *stats);

/* ---- sharded streaming receive (one process per GPU, SURVEY §8e raw single stream) ----
 * The receiver's state between blocks (StreamingReceiver fields): */
typedef struct amod_stream_state {
  int64_t block;                 /* next block to process                               */
  int64_t ac_pos, pre_pos, frame_end;
  double ac_p, ac_ra, ac_rb;
  int32_t state, ac_init, meta_received, chunk_size;
} amod_stream_state;
/* one demodulated window of a shard's trajectory and the state right after it */
typedef struct amod_stream_event {
  amod_stream_frame frame;       /* pos, end, window_len, decodeChunkFrame result       */
  amod_stream_state after;       /* after _resetToIdle, positioned at the next block     */
} amod_stream_event;
/* A shard holds stream samples [lo, hi) (host; lo a multiple of 8192, hi of 4096) and
 * owns blocks from own_lo (a multiple of 4096). start == NULL: it starts speculatively
 * at own_lo (IDLE, the scan resuming there) with the given metadata state; otherwise at
 * *start (the true state, e.g. rank 0). until_meta: stop after the first window whose
 * result makes the metadata state known (every window decoded as it comes). The run
 * covers blocks up to hi, every window it demodulates at pos >= own_lo is decoded
 * (payload rows of `stride` bytes), failed refinements go to fails as (block, pos)
 * pairs. ema[0] / ema[1]: the DC-removal state after sample own_lo - 1 / own_hi - 1
 * (own_hi a multiple of 8192; the neighbours' exactness check); *end: the state after the last block. Windows whose
 * runs agree on a post-reset state continue identically; amodem/shard.py merges the
 * shards' trajectories at such a window.                             */
int amod_stream_shard(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t lo, int64_t hi,
                      int64_t own_lo, int64_t own_hi, const amod_stream_state *start, int32_t meta_received, int32_t chunk_size,
                      int32_t until_meta, amod_stream_event *events, int64_t max_events, int64_t *nevents,
                      uint8_t *payload, int64_t stride, int64_t *fails, int64_t max_fails, int64_t *nfails,
                      double *ema, amod_stream_state *end);

/* ---- live streaming receive: StreamingReceiver.processAudioBlock (app.js:749-773) ----
 * One call per audio callback block (any length; the reference's ScriptProcessor hands
 * 4096 samples): DC removal, ring buffer, one step of the receiver's state machine.
 * When the step demodulates a window (_demodulateFrame, app.js:907-972), *has_frame = 1
 * and *frame holds it (decoded on the GPU, dispatched to the assembler before return).
 * Fed the blocks of a recorded stream, the frames equal amod_stream_receive's. */
typedef struct amod_live amod_live;
typedef struct amod_live_stats {
  int64_t total_written;       /* ringBuffer.totalWritten                             */
  int64_t frames_decoded, frame_errors; /* the receiver's counters                    */
  int64_t refine_fails;        /* _refineAndCollect false positives (back to idle)    */
  int64_t last_refine_fail;    /* preambleGlobalPos of the last one, or -1            */
  int64_t fine_host_positions; /* cross-correlation positions evaluated              */
} amod_live_stats;
/* assembler NULL: a private one (closed with the receiver) */
int amod_live_open(amod_ctx *ctx, const amod_cfg *cfg, amod_assembler *assembler, amod_live **out);
int amod_live_process_block(amod_live *lv, const float *samples, int64_t n, amod_stream_frame *frame,
                            int32_t *has_frame);
int amod_live_state(const amod_live *lv, amod_stream_state *state, amod_live_stats *stats);
/* positions of the failed refinements so far (up to max); returns their count */
int64_t amod_live_refine_fails(const amod_live *lv, int64_t *pos, int64_t max);
void amod_live_close(amod_live *lv);


/* deterministic synthetic payload (xorshift32, 4 bytes per step, little-endian) */
void amod_synth_payload(uint32_t seed, int32_t len, uint8_t *out);
/* nframes legacy frames of payload_len bytes each (seed 0x9E3779B9 ^ (first+i), name),
   laid out back to back in out; offsets/lengths filled; threads <= 0 -> hardware threads.
   Returns total samples (out NULL: sizing only). */
int64_t amod_synth_legacy_batch(const amod_cfg *cfg, int32_t nframes, int32_t first, int32_t payload_len,
                                const uint8_t *name, int32_t name_len, float *out, int64_t *offsets,
                                int32_t *lengths, int32_t threads);

#ifdef __cplusplus
}
#endif
#endif /* AMODEM_H */
