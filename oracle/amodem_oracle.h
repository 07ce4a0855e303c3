/*
 * amodem_oracle.h — CPU restatement of the playok/audio-modem receive path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker for the HIP
 * product in audio-modem_amd/: only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it. The product never links or calls it.
 *
 * Every function restates the reference's arithmetic in IEEE double with the
 * same operation order (compiled with -ffp-contract=off), so results are
 * bit-identical to modem.js running in V8. Pinned by the JSON fixtures in tests/golden/,
 * which were produced by the unmodified reference (tests/golden/gen_golden.js).
 * Citations are to /root/reference/modem.js unless noted.
 */
#ifndef AMODEM_ORACLE_H
#define AMODEM_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_PILOTS 32

typedef struct {
  int fft_size, cp_len, symbol_len, sample_rate, sub_start, sub_end;
  int npilots;
  int pilots[ORC_MAX_PILOTS];
} orc_cfg;

enum { ORC_BPSK = 0, ORC_QPSK = 1, ORC_QAM16 = 2 };

/* status codes: same numbering as include/amodem.h AMOD_* */
enum {
  ORC_OK = 0,
  ORC_E_PREAMBLE = 1,        /* 'Preamble not detected' */
  ORC_E_LOW_CORR = 2,        /* 'Preamble not detected (low correlation)' */
  ORC_E_SHORT_CE = 3,        /* 'Signal too short for CE' */
  ORC_E_NO_DATA = 4,         /* 'No data after CE' */
  ORC_E_DECODED_SHORT = 5,   /* 'Decoded data too short' */
  ORC_E_SHORT_HEADER = 6,    /* 'Decoded data too short for header' */
  ORC_E_INVALID_LEN = 7,     /* `Invalid data length: ${aux}` */
  ORC_E_META_SHORT = 8,      /* 'Metadata frame too short' */
  ORC_E_META_TRUNC = 9,      /* 'Metadata frame truncated' */
  ORC_E_CHUNK_SHORT = 10,    /* 'Data chunk frame too short' */
  ORC_E_CHUNK_TRUNC = 11,    /* 'Data chunk truncated' */
  ORC_E_FRAME_SHORT_CE = 12, /* 'Frame too short for CE' */
  ORC_E_UNKNOWN_TYPE = 13,   /* `Unknown frame type: 0x${aux.toString(16)}` */
};

typedef struct {
  int32_t status, preamble_idx, coarse_idx, frame_type, aux, nbytes;
  int32_t name_off, name_len, data_off, data_len;
  int32_t seq_num, total_chunks, total_size, chunk_size;
  uint32_t expected_crc, actual_crc;
  int32_t crc_valid, nbits;
  double fine_metric;
} orc_result;

/* configuration presets (modem.js:69-98); unknown names fall back to standard */
void orc_config(const char *name, orc_cfg *out);
int orc_num_data_subs(const orc_cfg *c);
int orc_bps(int mod);

/* primitives */
void orc_fft(double *re, double *im, int n, int inverse); /* modem.js:6-66, in place, ifft scaled */
double orc_seeded_next(double *state);                    /* modem.js:153-156 */
void orc_preamble1(const orc_cfg *c, float *out);         /* SYMBOL_LEN floats, modem.js:158-170 */
void orc_preamble2(const orc_cfg *c, float *out);         /* modem.js:172-184 */
void orc_ce_symbol(const orc_cfg *c, float *out, double *known_re); /* modem.js:186-200 */
void orc_const_point(int mod, int idx, double *re, double *im);     /* modem.js:107-131 */
int orc_demap(int mod, double re, double im);             /* index; modem.js:140-150 */
uint32_t orc_crc32(const uint8_t *d, size_t n);           /* modem.js:443-457 */
int orc_majority(const uint8_t *bits, int nbits, int n, uint8_t *out); /* modem.js:487-495 */
int orc_bits_to_bytes(const uint8_t *bits, int nbits, uint8_t *out);   /* modem.js:468-476 */
int orc_estimate_frame_samples(const orc_cfg *c, int payload, int mod, int rep); /* modem.js:863-874 */

/* receive chain stages */
void orc_dc_remove(const float *x, long n, float *out, double *state);
void orc_preprocess(const float *x, int n, float *out, double *mean, double *mx); /* modem.js:213-232 */
int orc_detect_preamble(const float *sig, int n, const orc_cfg *c);               /* modem.js:286-319 */
int orc_fine_timing(const float *sig, int n, const orc_cfg *c, int coarse, double *best); /* modem.js:567-588 */
void orc_estimate_channel(const float *ce, const orc_cfg *c, double *h_re, double *h_im); /* modem.js:421-440 */
/* per-symbol detail: fft bins, eq, phase for symbol s of data (len samples) */
void orc_symbol_detail(const float *data, int len, int s, const orc_cfg *c, const double *h_re,
                       const double *h_im, double *x_re, double *x_im, double *eq_re, double *eq_im,
                       double *phase);
int orc_demodulate(const float *data, int len, const orc_cfg *c, int mod, const double *h_re,
                   const double *h_im, uint8_t *bits_out); /* modem.js:365-418; returns nbits */

/* full entry points. bytes_out receives the decoded byte stream (after vote),
   capacity bytes_cap; returns status. modem.js:557-654 and 770-803 */
int orc_decode_received(const orc_cfg *c, const float *x, int n, int mod, int rep, orc_result *r,
                        uint8_t *bytes_out, int bytes_cap);
int orc_decode_chunk(const orc_cfg *c, const float *x, int n, int mod, int rep, orc_result *r,
                     uint8_t *bytes_out, int bytes_cap);
/* parse of an already-decoded byte stream (modem.js:805-849); legacy tail of 622-653 */
void orc_parse_bytes(const uint8_t *b, int nb, int legacy_allowed, orc_result *r);

/* transmit restatement (synthetic inputs only). Return sample count; out may be NULL to size. */
int orc_build_legacy(const orc_cfg *c, const uint8_t *data, int len, const uint8_t *name, int name_len,
                     int mod, int rep, float *out);         /* modem.js:498-555 */
int orc_build_meta(const orc_cfg *c, int total_chunks, int total_size, int chunk_size,
                   const uint8_t *name, int name_len, int mod, int rep, float *out); /* 666-692,758 */
int orc_build_chunk(const orc_cfg *c, const uint8_t *data, int len, int seq, int mod, int rep,
                    float *out);                            /* 694-714,763 */
int orc_build_test_signal(const orc_cfg *c, int mod, int rep, float *out); /* 914-973 */

/* deterministic recipes shared with tests/golden/gen_golden.js */
uint32_t orc_xs32(uint32_t s);
void orc_payload(uint32_t seed, int len, uint8_t *out);
void orc_add_noise(const float *in, int n, int snr_db, uint32_t seed, float *out);
/* same generator with an explicit signal/noise power divisor (test fixtures' `div`) */
void orc_add_noise_div(const float *in, int n, double div, uint32_t seed, float *out);

/* multi-threaded CPU baseline: decode nframes legacy frames laid out at offsets */
double orc_bench_decode(const orc_cfg *c, const float *x, const int64_t *off, const int32_t *len,
                        int nframes, int mod, int rep, int threads, int32_t *status_out,
                        uint32_t *crc_out);
double orc_bench_decode_chunk(const orc_cfg *c, const float *x, const int64_t *off, const int32_t *len,
                        int nframes, int mod, int rep, int threads, int32_t *status_out,
                        uint32_t *crc_out);

#ifdef __cplusplus
}
#endif
#endif
