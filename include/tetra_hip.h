/*
 * tetra_hip.h -- C ABI of libtetra_hip.so, the MI355X (gfx950) TETRA receive hot path.
 *
 * Drop-in boundary for the reference's demod + lower-MAC path (WizzardDr/TetraEar-BladeRF):
 *   tetraear/signal/processor.py  SignalProcessor            (processor.py:18-273)
 *   tetraear/core/decoder.py      TetraDecoder lower MAC      (decoder.py:140-295, 835-888)
 *   tetraear/core/protocol.py     parse_burst / CRC           (protocol.py:192-347)
 * plus the ETSI EN 300 392-2 receive chain the reference lacks (BASELINE.json north_star):
 *   polyphase FIR channel filter/resampler, RRC matched filter, Gardner timing recovery,
 *   differential decision with soft bits, descrambler, block deinterleaver, RCPC depuncture,
 *   K=5 rate-1/4 Viterbi, CRC-16.
 *
 * Conventions
 *   - Every entry point returns 0 on success or a negative TETRA_E* code; nothing aborts.
 *     tetra_last_error() returns the message of the last failure on that context.
 *   - Array arguments may be HOST or DEVICE pointers (the library asks HIP which); host arrays
 *     are staged through context-owned device buffers (those of up to 128 KB through a pinned
 *     host arena of the context, as async copies).  Calls with device arguments enqueue on the
 *     context's stream and return without waiting; calls that touch host memory return after
 *     their results are in host memory.
 *   - Complex arrays are interleaved (re, im).  "cf32" = complex64, "cf64" = complex128.
 *   - One context per host thread; a context is not thread-safe.  No allocation happens on a
 *     repeat call with sizes no larger than a previous call (workspaces are cached).
 */
#ifndef TETRA_HIP_H
#define TETRA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TETRA_ABI_VERSION 2

enum {
    TETRA_OK = 0,
    TETRA_E_INVALID = -1,   /* bad argument */
    TETRA_E_HIP = -2,       /* HIP runtime error */
    TETRA_E_NODEVICE = -3,  /* no usable gfx950 device */
    TETRA_E_NOMEM = -4
};

/* Sample formats of input arrays.  TETRA_SC16: interleaved int16 (I, Q), the BladeRF wire format,
 * scaled by 1/32768 as capture.py:241-269 does (exact in fp32); ETSI channel filter only. */
enum { TETRA_CF32 = 0, TETRA_CF64 = 1, TETRA_SC16 = 2 };
/* Real samples (float32 / float64), taken only by tetra_demod_dqpsk: the reference's
 * demodulate_dqpsk on a real array (processor.py:124-140 with real scalars). */
enum { TETRA_F32 = 3, TETRA_F64 = 4 };

typedef struct tetra_ctx tetra_ctx;

int tetra_abi_version(void);
/* Create a context on HIP device `device`; NULL on failure (see tetra_last_error(NULL)). */
tetra_ctx *tetra_create(int device);
void tetra_destroy(tetra_ctx *ctx);
const char *tetra_last_error(const tetra_ctx *ctx);
/* The context's hipStream_t; tetra_set_stream() makes the context enqueue on a caller stream. */
void *tetra_get_stream(tetra_ctx *ctx);
int tetra_set_stream(tetra_ctx *ctx, void *hip_stream);
int tetra_synchronize(tetra_ctx *ctx);
/* Device name / arch of the context's device (e.g. "gfx950"). */
int tetra_device_arch(tetra_ctx *ctx, char *buf, size_t n);

/* Per-stage device timing: when enabled, every kernel stage is bracketed by HIP events on the
 * context stream.  tetra_profile_read() synchronizes, then returns the accumulated milliseconds
 * and launch counts per stage since the previous read (names NUL-separated, in first-seen order). */
int tetra_profile(tetra_ctx *ctx, int enable);
/* Diagnostic: the channel filter's HBM read pattern without its arithmetic (rows workgroups, one
 * row of row_bytes each, 16-B loads; lds_bytes of LDS per workgroup caps the residency like the
 * real kernel's).  Device pointer x; timed under the "read_floor" profile stage. */
int tetra_read_floor(tetra_ctx *ctx, const void *x, size_t rows, size_t row_bytes, size_t lds_bytes);
int tetra_profile_read(tetra_ctx *ctx, char *names, size_t names_len, double *ms, int64_t *count,
                       int max_stages, int *n_stages);
/* Diagnostic: launch the one-wave marker kernel k_region_mark(tag) on the context stream.  bench.py
 * brackets its timed steps with tag 1 / tag 2, so rocprofv3 traces and counter passes of the bench
 * command can select the timed launches by dispatch order (tools/pmc_summary.py). */
int tetra_mark(tetra_ctx *ctx, int tag);

/* =====================================================================================
 * Compat demod -- bit-compatible with SignalProcessor (processor.py:221-273) in its default
 * (sequential) form; the opt-in latency mode (TETRA_COMPAT_BLOCKED) is within fp32 noise only
 * ===================================================================================== */

/* Filter design and control decisions are made by the host (the same scipy.signal design calls
 * the reference makes: cheby1/sosfilt_zi for decimate, butter/lfilter_zi for filter_signal);
 * the plan carries them to the device.  Field-by-field:                                     */
typedef struct tetra_compat_plan {
    int32_t q;            /* decimation factor (processor.py:249); <= 1: decimation stage skipped */
    int32_t dec_f64;      /* 0: decimate in complex64 arithmetic (cf32 input), 1: complex128 */
    int32_t filt;         /* 1: filtfilt runs (len > padlen 15); 0: filter_signal returned input */
    int32_t ntaps;        /* butter(4) -> 5 */
    int32_t sps;          /* int(rate/18000) (processor.py:183) */
    int32_t phase_step;   /* max(1, sps//8) (processor.py:194) */
    int32_t flags;        /* TETRA_COMPAT_*: 0 = scipy's sequential order (bit-exact), BLOCKED = latency mode */
    int32_t reserved;
    double fs_dec;        /* sample rate after decimation: time base of frequency_shift */
    float sos_f32[24];    /* cheby1(8, 0.05, 0.8/q) SOS [4][6] as complex64 real parts */
    float zi_f32[8];      /* sosfilt_zi in complex64 */
    double sos_f64[24];
    double zi_f64[8];
    double b[8], a[8];    /* butter(4, cutoff) */
    double lzi[8];        /* lfilter_zi(b, a) */
    double thr[4];        /* -5*pi/8, -3*pi/8, 3*pi/8, 5*pi/8 as Python evaluates them */
} tetra_compat_plan;

/* tetra_compat_plan.flags.  The decimator and filtfilt of tetra_demod_compat run sequentially in
 * time by default (0, or TETRA_COMPAT_SEQUENTIAL): scipy's exact operation order, bit-identical to
 * the reference.  TETRA_COMPAT_BLOCKED opts into the latency mode: tiles of 256 (decimator) / 128
 * (filtfilt) samples recursed in parallel, their start states composed in float64, for C <= 64
 * channels, q <= 16 and N + 54 <= 262144 samples (TETRA_E_INVALID outside those limits); ~40x lower
 * latency for one channel but NOT bit-exact: the decimator ends up to ~1.5e-5 from scipy's fp32
 * state near the chunk start, so a decision whose phase margin is ~1e-6 rad can flip (measured: 3 in
 * 1.6 M symbols).  The component entry point tetra_decimate is always sequential. */
#define TETRA_COMPAT_SEQUENTIAL 1   /* the scipy-exact sequential passes (the default) */
#define TETRA_COMPAT_BLOCKED    2   /* the time-blocked latency mode (opt-in, not bit-exact) */

/* Host-only (no device needed): the kernels tetra_demod_compat would run for `plan` on a [C][N]
 * batch, as TETRA_FORM_* bits in *forms. */
#define TETRA_FORM_DEC_BLOCKED  1   /* decimate: time-blocked (else scipy's sequential order) */
#define TETRA_FORM_LF_BLOCKED   2   /* filtfilt: time-blocked (else scipy's sequential order) */
#define TETRA_FORM_POW_PREPASS  4   /* extract_symbols: |y|^2 first in parallel (exact either way) */
int tetra_compat_forms(const tetra_compat_plan *plan, size_t C, size_t N, int32_t *forms);

/* Fused process() over a batch of C equal-length chunks.
 *   iq        [C][N] complex, format iq_fmt (TETRA_CF32 for SC16-derived capture data)
 *   mix_c     [C] imaginary part of (-1j*2*pi*freq_offset) per channel (processor.py:98-99)
 *   mix_on    [C] 1 where freq_offset != 0 (processor.py:260)
 *   soft      [C][smax] complex128: the `.symbols` attribute (processor.py:268)
 *   hard      [C][smax] uint8: process() return value; hard count = max(0, nsym-1)
 *   nsym      [C] number of soft symbols per channel
 *   soft_f32  set to 1 when `.symbols` is complex64 in the reference (no filter, no mixer)
 * smax must be >= the symbol count the plan implies (tetra_compat_symbols()). */
int tetra_demod_compat(tetra_ctx *ctx, const tetra_compat_plan *plan, const void *iq, int iq_fmt,
                       size_t C, size_t N, const double *mix_c, const uint8_t *mix_on,
                       void *soft, uint8_t *hard, int32_t *nsym, size_t smax, int32_t *soft_f32);
/* Number of soft symbols process() yields for N input samples under `plan`. */
int64_t tetra_compat_symbols(const tetra_compat_plan *plan, size_t N);
/* Host-only: the latency mode's state-transition tables.  which = 0 / 1: the time-blocked
 * decimator's Phi^(2^r), r = 0..9, row-major 8 x 8 float64 each (Phi = A^256, A the 4-section
 * cascade's one-sample zero-input transition) from the plan's complex64 / complex128 SOS, 640
 * doubles; which = 2: the time-blocked filtfilt's Psi^(2^r) (Psi = B^128, B lfilter's one-sample
 * transition of its 4 states), 160 doubles. */
int tetra_compat_blocked_table(const tetra_compat_plan *plan, int which, double *table);

/* Component entry points, one per SignalProcessor method (each over C rows of length N). */
/* scipy.signal.decimate(x, q) as called at processor.py:254: out [C][ceil(N/q)] in iq_fmt. */
int tetra_decimate(tetra_ctx *ctx, const tetra_compat_plan *plan, const void *iq, int iq_fmt,
                   size_t C, size_t N, void *out);
/* frequency_shift (processor.py:85-100): out [C][N] complex128. */
int tetra_frequency_shift(tetra_ctx *ctx, const void *iq, int iq_fmt, size_t C, size_t N,
                          const double *mix_c, double fs, void *out);
/* filter_signal's filtfilt (processor.py:78-79): out [C][N] complex128; needs N > 3*ntaps. */
int tetra_filtfilt(tetra_ctx *ctx, const tetra_compat_plan *plan, const void *iq, int iq_fmt,
                   size_t C, size_t N, void *out);
/* extract_symbols (processor.py:168-219): sym [C][smax] in iq_fmt, nsym [C], best phase [C]. */
int tetra_extract_symbols(tetra_ctx *ctx, const void *x, int fmt, size_t C, size_t N, int sps,
                          int phase_step, void *sym, int32_t *nsym, int32_t *best_phase, size_t smax);
/* demodulate_dqpsk (processor.py:102-166): hard [C][S-1] for C rows of S symbols in TETRA_CF32 /
 * TETRA_CF64, or real rows in TETRA_F32 / TETRA_F64. */
int tetra_demod_dqpsk(tetra_ctx *ctx, const void *sym, int fmt, size_t C, size_t S,
                      const double *thr4, uint8_t *hard);

/* =====================================================================================
 * Compat lower MAC -- TetraDecoder.decode / find_sync / parse_burst (decoder.py, protocol.py)
 * ===================================================================================== */

#define TETRA_MAX_SYNC 16
/* Per-sync record written by tetra_lmac_compat (int32 fields). */
enum {
    TETRA_F_POS = 0,      /* sync position (bit index of the training sequence) */
    TETRA_F_START,        /* pos - 216 (decoder.py:865) */
    TETRA_F_VALID,        /* 1 if the frame is sliced (start >= 0 and start//2+255 <= S) */
    TETRA_F_NBITS,        /* len(bits[start:start+510]) (decoder_frame needs 510) */
    TETRA_F_NUMBER,       /* start // 510 (decoder.py:881) */
    TETRA_F_BTYPE,        /* BurstType value: 2 NormalDownlink, 5 Synchronization */
    TETRA_F_CRC,          /* parse_burst crc_ok */
    TETRA_F_HDR,          /* (pdu_type << 2) | encryption_mode (decoder.py:906-909) */
    TETRA_F_FIELDS = 8
};

/* Batched decode() lower MAC for C symbol streams.
 *   sym       [C][stride] int64 symbols (0..3, or 0..7 for the 8-PSK branch)
 *   nsym      [C] stream lengths
 *   k_of_max  [23] sync count threshold as a function of the stream's best correlation count,
 *             -1 for "no sync" (the 0.90/0.85/0.80/adaptive cascade, decoder.py:845-857,
 *             tabulated by the host)
 *   nsync     [C]; rec [C][TETRA_MAX_SYNC][TETRA_F_FIELDS]
 *   frame_bits[C][TETRA_MAX_SYNC][510] = bits[start:start+510]  (decode_frame 'bits')
 *   burst_bits[C][TETRA_MAX_SYNC][510] = bits of mapped[start//2:+255] (parse_burst input)  */
int tetra_lmac_compat(tetra_ctx *ctx, const int64_t *sym, const int32_t *nsym, size_t C, size_t stride,
                      const int8_t *k_of_max, int32_t *nsync, int32_t *rec, uint8_t *frame_bits,
                      uint8_t *burst_bits);
/* symbols_to_bits (decoder.py:140-169): bits [2S] int64, mapped [S] int64. */
int tetra_symbols_to_bits(tetra_ctx *ctx, const int64_t *sym, size_t S, int64_t *bits, int64_t *mapped);
/* find_sync main scan (decoder.py:226-259) at integer count threshold kthr:
 * pos [maxpos], *npos hits, *maxc = max evaluated correlation count. */
int tetra_find_sync(tetra_ctx *ctx, const uint8_t *bits, size_t nbits, int kthr, int64_t *pos,
                    int maxpos, int32_t *npos, int32_t *maxc);
/* Pattern match counts (the np.sum(window == pattern) of decoder.py:239 / protocol.py:262):
 * counts[f] = #{j < 22 : bits[f][offset+j] == pattern22[j]} over F rows of L bytes. */
int tetra_match_count(tetra_ctx *ctx, const uint8_t *bits, size_t F, size_t L, const uint8_t *pattern22,
                      size_t offset, int32_t *counts);
/* parse_burst over F bursts of 255 symbols (protocol.py:192-244): btype [F], crc_ok [F],
 * bits [F][510] burst bits (training sequence/data are slices of these). */
int tetra_parse_bursts(tetra_ctx *ctx, const int64_t *sym, size_t F, int32_t *btype, uint8_t *crc_ok,
                       uint8_t *bits);
/* _calculate_crc16 over F rows of L bits (reversed != 0: payload reversed): crc [F]. */
int tetra_crc16(tetra_ctx *ctx, const uint8_t *bits, size_t F, size_t L, int reversed, uint16_t *crc);
/* _check_crc over F rows of L bits: ok [F]. */
int tetra_check_crc(tetra_ctx *ctx, const uint8_t *bits, size_t F, size_t L, uint8_t *ok);

/* MAC PDU header extraction of TetraProtocolParser.parse_mac_pdu (protocol.py:349-596; SURVEY.md
 * §8f rank 4) over F frames of data bits, one byte per bit (any nonzero byte reads as 1, in the
 * header fields and the data bytes alike), one row of `stride` bytes each, nbits[f] valid.
 * Stateless per frame: the fragment buffer, the MCC/MNC/colour-code state and the statistics are
 * applied in order by the host (tetraear.core.protocol.parse_mac_pdu_batch).
 *   fields [F][TETRA_MAC_FIELDS] (below); data [F][data_stride] = BitArray(data bits).tobytes()
 *   (MSB first, last byte zero-padded), data_stride >= (stride + 7) / 8. */
enum {
    TETRA_MAC_STATUS = 0,   /* 0 PDU; 1 None, no state touched (len < 8, truncated address/length,
                               length check protocol.py:433/525, short SYSINFO); 2 None after the
                               SYSINFO state write (MCC outside 200..799 or MNC > 999, :489-494) */
    TETRA_MAC_PTYPE,        /* PDUType value: 0 RESOURCE, 1 FRAG, 2 END (header 3), 3 BROADCAST (header 2) */
    TETRA_MAC_MODE,         /* (bits[2] << 1) | bits[3] (:389) */
    TETRA_MAC_FILL,         /* bits[4] (RESOURCE, FRAG, END), else 0 */
    TETRA_MAC_ADDR,         /* 24-bit address (RESOURCE), else -1 */
    TETRA_MAC_LENGTH,       /* 6-bit length indicator (RESOURCE, END), else 0 */
    TETRA_MAC_DATA_BITS,    /* number of data bits packed into data[f] */
    TETRA_MAC_SYSINFO,      /* 1 if the SYSINFO MCC/MNC/colour code below were read (:482-485) */
    TETRA_MAC_MCC,
    TETRA_MAC_MNC,
    TETRA_MAC_CC,
    TETRA_MAC_FIELDS = 12
};
int tetra_mac_headers(tetra_ctx *ctx, const uint8_t *bits, const int32_t *nbits, size_t F, size_t stride,
                      int32_t *fields, uint8_t *data, size_t data_stride);

/* Signal-present / AFC gate of the capture loop (/root/reference/tetraear/ui/modern.py:1952-2028,
 * SURVEY.md §8f rank 1), per channel on the 2048-point Hann spectrum of its first 2048 samples
 * (the k_waterfall row, fused): centre band of int(25000 / (fs / 2048)) bins around bin 1024, noise
 * floor from the bins 10 beyond it on both sides, present iff snr > 15 dB and peak > -70 dBFS and
 * peak - band mean > 3 dB, AFC offset = the peak bin's frequency when present.  stats [C][FIELDS]
 * (host or device); power [C][2048] the dB rows or NULL; mixer_coef / mixer_on [C] (or NULL) the
 * offset as tetra_demod_compat's mixer arguments (-2 pi f, f != 0), so process() runs on the gate's
 * AFC with no host round trip.  N < 2048: no detection (all zero). */
enum {
    TETRA_GATE_VALID = 0,     /* 1 when a centre band exists (N >= 2048 and >= 2 band bins) */
    TETRA_GATE_SIGNAL,        /* mean dB of the centre band */
    TETRA_GATE_PEAK,          /* max dB of the centre band */
    TETRA_GATE_PEAK_BIN,      /* its first index (0..2047, fftshifted) */
    TETRA_GATE_PEAK_FREQ,     /* its frequency fftshift(fftfreq(2048, 1/fs))[bin], Hz */
    TETRA_GATE_NOISE,         /* noise floor (mean dB outside the band +- 10 bins, -100 if none) */
    TETRA_GATE_SNR,           /* signal - noise */
    TETRA_GATE_ABOVE,         /* peak - signal */
    TETRA_GATE_PRESENT,       /* 1: signal present (the three thresholds) */
    TETRA_GATE_AFC,           /* the freq_offset process() gets: PEAK_FREQ when present, else 0 */
    TETRA_GATE_FIELDS = 10
};
int tetra_afc_gate(tetra_ctx *ctx, const void *iq, int iq_fmt, size_t C, size_t N, double fs, float *power,
                   double *stats, double *mixer_coef, uint8_t *mixer_on);

/* The scanner's TETRA signal detector over a batch of candidate channels (SURVEY.md §8f rank 2;
 * replaces the per-sample Python loops of /root/reference/tetraear/signal/scanner.py:42-147 and
 * 204-231): per channel of iq [C][N] (TETRA_CF32 / TETRA_CF64) the counts the detector's decisions
 * are made from -- the pi/4-DQPSK cluster test over consecutive samples, the best 31-bit match of
 * sync_pattern (bit j of the word = pattern bit j) over the bits of the samples strided by
 * `downsample`, and the mean powers of the chunk and of its five equal windows -- into
 * stats [C][TETRA_SCAN_FIELDS] (host or device).  At most 131072 sync bits per channel. */
enum {
    TETRA_SCAN_MOD_MATCHES = 0,   /* phase differences within pi/8 of a multiple of pi/4 in [-pi, 3pi/4] */
    TETRA_SCAN_MOD_DIFFS,         /* N - 1 */
    TETRA_SCAN_SYNC_MATCHES,      /* best match count (0..31) over the window starts */
    TETRA_SCAN_SYNC_WINDOWS,      /* window starts searched: max(0, nbits - 31) */
    TETRA_SCAN_SYNC_BITS,         /* bits: strided samples - 1 */
    TETRA_SCAN_POWER,             /* mean |x|^2 */
    TETRA_SCAN_POWER_W0,          /* mean |x|^2 of window i = [i (N/5), (i+1) (N/5)), i = 0..4 */
    TETRA_SCAN_FIELDS = TETRA_SCAN_POWER_W0 + 5
};
int tetra_scan_detect(tetra_ctx *ctx, const void *iq, int iq_fmt, size_t C, size_t N, int downsample,
                      uint32_t sync_pattern, double *stats);

/* =====================================================================================
 * ETSI EN 300 392-2 receive chain (north star; no reference counterpart)
 * ===================================================================================== */

/* Receiver design (filled by the host: tetraear.signal.etsi.etsi_plan).  Stage 1: L1-tap FIR
 * decimating by q1 (fs -> fs1 = fs / q1); stage 2: RRC (0.35) polyphase prototype of Lp taps at
 * up * fs1 = 4 * down * 18 kHz, resampled x up/down to 72 kHz (4 samples/symbol); then timing.
 *   2.4 MSps: q1 = 10, L1 = 48, 3/10, Lp = 321 -- the canonical plan, run by the fused per-wave
 *             kernels (k_chanfilt_r / k_chanfilt);
 *   any other plan with q1 <= 13, L1 <= 64, Lp <= 4096 and (Lp - 1) / up <= 256 (e.g. the
 *             reference CLI's 1.8-2.4 MSps in 0.1 MHz steps, modern.py:5518-5519, 5630-5638): the
 *             generic-rate channel filter k_chanfilt_g (y through HBM) + k_timing.
 * flags bit 0 (TETRA_ETSI_FORCE_GENERIC): run a canonical plan on the generic kernel too (tests). */
#define TETRA_ETSI_FORCE_GENERIC 1
typedef struct tetra_etsi_plan {
    int32_t q1, L1, Lp, up, down;
    float gain;           /* block-Gardner loop gain */
    float soft_scale;     /* int8 soft-bit scale: soft = rint(x * soft_scale / mean|d|) */
    int32_t flags;
    float h1[64];
    float hp[4096];
} tetra_etsi_plan;

#define TETRA_ETSI_MAXB 8    /* bursts per channel chunk */
#define TETRA_ETSI_MAXJ 16   /* coded blocks per channel chunk */
/* block kinds */
enum { TETRA_SCH_F = 0, TETRA_SCH_HD = 1, TETRA_BSCH = 2 };
/* burst kinds */
enum { TETRA_NDB_N = 0, TETRA_NDB_P = 1, TETRA_SB = 2 };

/* M1 (240 kHz samples), M2 (72 kHz samples) and the symbol capacity smax for N input samples. */
int tetra_etsi_lengths(const tetra_etsi_plan *plan, size_t N, int64_t *M1, int64_t *M2, int64_t *smax);
/* Channel filter + RRC resampler: iq [C][N] cf32 -> y [C][M2] cf32. */
int tetra_etsi_chanfilt(tetra_ctx *ctx, const tetra_etsi_plan *plan, const void *iq, size_t C, size_t N, void *y);
/* Timing recovery + differential decision: y [C][M2] ->
 *   soft [C][smax] cf32 symbol-spaced samples (the ETSI `.symbols`), softbits [C][2*smax] int8
 *   (>0: bit 0), hard [C][smax] dibit symbols 0..3 (count nsym-1), nsym [C],
 *   diag [C][4] (timing phase, final Gardner correction, CFO rotation re/im) or NULL.
 *   Entries past a channel's nsym (symbols) and nsym-1 (soft bits, dibits) are unspecified.
 *   TETRA_TIMING_PROBE=1 (diagnostic): diag holds four 32-bit wall-clock stamps per channel instead. */
int tetra_etsi_timing(tetra_ctx *ctx, const tetra_etsi_plan *plan, const void *y, size_t C, size_t M2,
                      void *soft, int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax, float *diag);
/* tetra_etsi_timing for the wideband chain's chunks, with the Oerder-Meyr class sums formed from
 * the resampler's group partials om (tetra_channelize_om) instead of a pass over y: y [C][M2] is
 * C / nchunk carrier rows of nchunk consecutive chunks, om [C / nchunk][ngrp] float4 the rows'
 * partials over groups of U outputs (U a multiple of 4, <= 64; ngrp U >= nchunk M2; M2 a multiple
 * of 4).  The class sums follow oracle/etsi_oracle.c eo_om_grouped (a summation order of the same
 * |y|^2 class sums; same outputs as tetra_etsi_timing otherwise; no reference counterpart). */
int tetra_etsi_timing_om(tetra_ctx *ctx, const tetra_etsi_plan *plan, const void *y, size_t C, size_t M2,
                         const void *om, size_t nchunk, size_t ngrp, int U, void *soft, int8_t *softbits,
                         uint8_t *hard, int32_t *nsym, size_t smax, float *diag);
/* tetra_etsi_timing over overlapping chunks of M carrier rows y [M][rowlen]: output row k nchunk + c
 * is the timing of y[k][c stride, min(c stride + len, rowlen)) (len > stride: consecutive chunks
 * share len - stride samples, so a burst that straddles one chunk's end lies whole in it -- the
 * wideband chain's seams lose no burst).  om: NULL (each chunk's own Oerder-Meyr pass over y) or
 * the rows' resampler partials [M][ngrp] float4 as in tetra_etsi_timing_om (stride a multiple of 4,
 * ngrp U >= rowlen).  smax >= len / 4 + 2.  Outputs as tetra_etsi_timing with C = M nchunk; a
 * chunk's outputs are the oracle's timing of its samples (no reference counterpart: the reference
 * demodulates one narrowband capture at a time, tetraear/signal/processor.py:253-331). */
int tetra_etsi_timing_chunks(tetra_ctx *ctx, const tetra_etsi_plan *plan, const void *y, size_t M, size_t rowlen,
                             size_t nchunk, size_t stride, size_t len, const void *om, size_t ngrp, int U, void *soft,
                             int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax, float *diag);
/* Fused demod (chanfilt + timing) over a batch. */
int tetra_demod_etsi(tetra_ctx *ctx, const tetra_etsi_plan *plan, const void *iq, size_t C, size_t N,
                     void *soft, int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax, float *diag);
/* The same two entry points for an explicit input format (TETRA_CF32 or TETRA_SC16); the
 * format-less forms above take cf32. */
int tetra_etsi_chanfilt_fmt(tetra_ctx *ctx, const tetra_etsi_plan *plan, const void *iq, int iq_fmt, size_t C,
                            size_t N, void *y);
int tetra_demod_etsi_fmt(tetra_ctx *ctx, const tetra_etsi_plan *plan, const void *iq, int iq_fmt, size_t C,
                         size_t N, void *soft, int8_t *softbits, uint8_t *hard, int32_t *nsym, size_t smax,
                         float *diag);
/* Differential decision on n given symbol-spaced samples x (TETRA_CF32 / TETRA_CF64): hard [n-1]
 * dibits by EN 300 392-2 Table 5.1 (the fused demod's decision, no CFO rotation).  Replaces the
 * reference's demodulate_dqpsk (/root/reference/tetraear/signal/processor.py:102-166) in ETSI mode,
 * whose shifted decision regions SURVEY.md §0.3 documents. */
int tetra_etsi_decide(tetra_ctx *ctx, const void *x, int iq_fmt, size_t n, uint8_t *hard);
/* The channel-filter kernel a demod (fused != 0) or chanfilt call on N-sample rows of iq_fmt runs:
 * its symbol name and static LDS bytes per workgroup (the occupancy the bench's read floor mimics). */
int tetra_etsi_kernel_info(tetra_ctx *ctx, const tetra_etsi_plan *plan, int iq_fmt, size_t N, int fused, char *name,
                           size_t name_len, int64_t *lds_bytes);
/* Cell configuration: scrambling code init per channel ((MCC<<20|MNC<<6|CC)<<2|3). */
int tetra_etsi_set_cells(tetra_ctx *ctx, const uint32_t *scramb_init, size_t C);
/* Lower MAC: burst sync + descramble + deinterleave + depuncture + Viterbi + CRC per channel.
 *   nburst [C], bursts [C][TETRA_ETSI_MAXB][2] (start bit, burst kind),
 *   nblock [C], blocks [C][TETRA_ETSI_MAXJ][4] (block kind, crc_ok, burst index, block index),
 *   type1 [C][TETRA_ETSI_MAXJ][268] decoded type-1 bits. */
int tetra_lmac_etsi(tetra_ctx *ctx, const int8_t *softbits, const uint8_t *hard, const int32_t *nsym,
                    size_t C, size_t smax, int32_t *nburst, int32_t *bursts, int32_t *nblock,
                    int32_t *blocks, uint8_t *type1);
/* Lower MAC with cell acquisition: the same outputs as tetra_lmac_etsi, without a configured cell.
 * cell_init [C] (in/out, host or device) holds each channel's scrambling init before the chunk
 * (3 = colour code 0 / not yet acquired).  The chunk's BSCH blocks are decoded first (colour code
 * 0, as every receiver must before it knows the cell); the last CRC-good one sets the channel's
 * extended colour code from its type-1 bits -- MAC-SYNC colour code bits 4..9, D-MLE-SYNC MCC bits
 * 31..40 and MNC bits 41..54 (EN 300 392-2 §21.4.4.2, §18.4.2.1) -- and the SCH/F / SCH/HD blocks
 * are then descrambled with it (§8.2.5.2).  cell_init returns the updated inits, so a stream of
 * chunks keeps the cell it acquired, as the reference parser keeps the MCC/MNC/colour code it
 * reads from a SYSINFO broadcast (/root/reference/tetraear/core/protocol.py:479-485).  The
 * scrambling table is cached per channel in the context and regenerated on the device only for
 * channels whose init changed. */
int tetra_lmac_etsi_acquire(tetra_ctx *ctx, const int8_t *softbits, const uint8_t *hard, const int32_t *nsym,
                            size_t C, size_t smax, uint32_t *cell_init, int32_t *nburst, int32_t *bursts,
                            int32_t *nblock, int32_t *blocks, uint8_t *type1);
/* ---------------------------------------------------------------- streaming (one continuous capture)
 * The reference's callers stream a continuous capture in chunks (modern.py:1901-1919,
 * continuous_capture.py:20); these entry points decode consecutive chunks of each channel as ONE
 * symbol stream, so no burst is lost at a chunk seam (oracle/etsi.py: Stream restates them).
 *   1. tetra_etsi_stream_window: where chunk k's channel-filter window starts.  The window re-reads
 *      the previous chunk's last samples from s, a multiple of P = q1 * down input samples, so its
 *      filter phases equal a run over the whole capture; yoff = its first new 72 kHz output.
 *   2. tetra_demod_etsi_stream: the fused demod over the window (rows of `ld` samples: a capture
 *      resident as [C][ld] is windowed in place) with each channel's timing loop carried in track.
 *   3. tetra_lmac_etsi_stream: the lower MAC over rows that hold the previous chunk's unconsumed
 *      dibits in front of the new ones; the greedy burst scan resumes at the bit it stopped at. */
typedef struct tetra_etsi_track {
    float base;       /* next symbol's Gardner base position, 72 kHz samples from the end of the last chunk's outputs */
    float delta;      /* block-Gardner loop offset */
    float prev_re, prev_im;   /* the last symbol of the previous chunk (dibit 0 of the next spans the seam) */
    int32_t acquired;         /* 0: the next chunk acquires the phase (Oerder-Meyr) and starts a new chain */
    int32_t reserved[3];
} tetra_etsi_track;
#define TETRA_ETSI_RESERVE 256   /* dibits ahead of a streaming output row (the lower MAC's carried tail) */
#define TETRA_ETSI_MARGIN 8      /* 72 kHz samples a window re-computes before its first new output */

/* Host-only window arithmetic: for a stream of x_total samples already received (y_done 72 kHz
 * outputs produced) and a next chunk of n samples: *s = the window's first sample (global index),
 * *W = its length (x_total + n - s), *yoff = the window index of output y_done, *y_done_next. */
int tetra_etsi_stream_window(const tetra_etsi_plan *plan, int64_t x_total, int64_t y_done, int64_t n, int64_t *s,
                             int64_t *W, int64_t *yoff, int64_t *y_done_next);
/* Fused demod of one window per channel: iq points at the window's first sample of channel 0, rows
 * ld samples apart (ld >= W, a multiple of 4 for SC16); track [C] (in/out, host or device).  Outputs
 * as tetra_demod_etsi_fmt, rows `ostride` symbols apart with capacity smax: with track[c].acquired,
 * symbol 0 is the carried last symbol of the previous chunk, so the nsym-1 dibits start with the one
 * across the seam. */
int tetra_demod_etsi_stream(tetra_ctx *ctx, const tetra_etsi_plan *plan, const void *iq, int iq_fmt, size_t C,
                            size_t ld, size_t W, int yoff, tetra_etsi_track *track, void *soft, int8_t *softbits,
                            uint8_t *hard, int32_t *nsym, size_t smax, size_t ostride, float *diag);
/* Lower MAC over streaming rows: row c of hard (softbits) is `stride` dibits (2 stride bytes); this
 * chunk's nsym[c]-1 dibits start at TETRA_ETSI_RESERVE, the previous chunk's tail is in front of
 * them and lead[c] (in/out) is the row bit the scan starts at (2 * TETRA_ETSI_RESERVE for a new
 * stream).  After the scan the unconsumed dibits (from the first bit not examined) are copied in
 * front of TETRA_ETSI_RESERVE in next_soft / next_hard (the rows the next chunk's demod writes;
 * they may be these rows) and lead[c] set for the next chunk.  bursts[.][0] is the burst's start
 * bit relative to this chunk's first new dibit (negative: it began in the carried tail).
 * cell_init: NULL (configured cells) or the acquisition state, as tetra_lmac_etsi_acquire. */
int tetra_lmac_etsi_stream(tetra_ctx *ctx, const int8_t *softbits, const uint8_t *hard, const int32_t *nsym,
                           size_t C, size_t stride, int32_t *lead, int8_t *next_soft, uint8_t *next_hard,
                           uint32_t *cell_init, int32_t *nburst, int32_t *bursts, int32_t *nblock, int32_t *blocks,
                           uint8_t *type1);

/* The ETSI receiver's AFC mixer on a streaming window: out [C][N] cf32 = iq (cf32 rows ld samples
 * apart) x exp(-j 2 pi f (n0 + n) / fs), n0 = the window's first sample in the capture (frequency_shift's
 * float64 arithmetic, processor.py:85-100, with one continuous phase across windows); mix_c [C] as
 * tetra_demod_compat's (the imaginary part of -1j*2*pi*f). */
int tetra_etsi_mix(tetra_ctx *ctx, const void *iq, size_t C, size_t ld, size_t N, const double *mix_c, double fs,
                   int64_t n0, void *out);

/* Component: decode F type-5 soft blocks of one kind (K = 432/216/120): type1 [F][n1], crc_ok [F]. */
int tetra_etsi_decode_blocks(tetra_ctx *ctx, const int8_t *soft5, size_t F, int kind,
                             const uint32_t *scramb_init, uint8_t *type1, uint8_t *crc_ok);
/* Component: encode F type-1 blocks (CRC, tail, RCPC 2/3, interleave, scramble): type5 [F][K]. */
int tetra_etsi_encode_blocks(tetra_ctx *ctx, const uint8_t *type1, size_t F, int kind,
                             const uint32_t *scramb_init, uint8_t *type5);

/* Synthetic capture generator (device side; bench.py and tests).  Per channel: a continuous
 * downlink of coded bursts (1/2 normal-n, 1/4 normal-p, 1/4 sync), pi/4-DQPSK + RRC(0.35) at fs,
 * random carrier phase, CFO uniform in [-cfo_max, cfo_max] Hz, AWGN at Es/N0 = snr_db (no noise if
 * snr_db >= 200), SC16 quantisation.  Each sync burst's BSCH carries a SYNC PDU of the channel's
 * cell (colour code at type-1 bits 4..9, MCC 31..40, MNC 41..54, the rest random).  Outputs: iq [C][N] cf32, cell_init [C] scrambling inits,
 * and optionally kinds [C][NB] burst kinds, payload [C][NB][2][268] type-1 bits (zero-padded),
 * t0 [C] symbol time of sample 0; NB = tetra_synth_bursts_per_channel(N, fs). */
int tetra_synth_bursts_per_channel(size_t N, double fs);
int tetra_synth_etsi(tetra_ctx *ctx, size_t C, size_t N, double fs, uint64_t seed, float snr_db, float cfo_max,
                     void *iq, uint32_t *cell_init, int32_t *kinds, uint8_t *payload, double *t0);

/* ---------------------------------------------------------------- wideband channeliser (C3)
 * A fs = 20 MSps capture -> M carriers at fs/M spacing (polyphase filter bank, D = M/4, rocFFT)
 * -> per-carrier RRC(0.35) resampler fs/D -> 72 kHz (up/down) = the ETSI timing stage's input
 * (tetra_etsi_timing).  Replaces tuning the SDR to one carrier per capture (the reference's
 * capture loop, /root/reference/tetraear/ui/modern.py:1886-1887 feeds one 2.4 MSps carrier
 * into SignalProcessor.process); SURVEY.md §8d config C3.  Host pointers h, g. */
typedef struct tetra_wb_plan {
    int32_t M;           /* carriers = FFT length (800) */
    int32_t D;           /* decimation, M / 4 (200): carrier rate fs / D */
    int32_t P;           /* prototype taps per branch, 1..8 (L = M * P) */
    int32_t up, down;    /* carrier resampler fs/D -> 72 kHz (18 / 25) */
    int32_t Lg;          /* resampler taps, a multiple of up */
    double fs;           /* wideband rate */
    const float *h;      /* prototype lowpass [M * P] (unity DC gain) */
    const float *g;      /* resampler RRC at up * fs / D [Lg] */
} tetra_wb_plan;

/* nblk filter-bank output blocks and n72 resampler outputs per carrier for Nw input samples. */
int tetra_wb_lengths(const tetra_wb_plan *plan, size_t Nw, int64_t *nblk, int64_t *n72);
/* x [Nw] cf32 -> y [M][n_keep] cf32 at 72 kHz (first n_keep <= n72 outputs of each carrier; a
 * carrier's row is then n_keep / M2 timing chunks of M2 samples for tetra_etsi_timing). */
int tetra_channelize(tetra_ctx *ctx, const tetra_wb_plan *plan, const void *x, size_t Nw, void *y, size_t n_keep);
/* tetra_channelize that also leaves om [M][ceil(n_keep / up)] float4: per carrier and group of up
 * consecutive outputs, the Oerder-Meyr class partials (sum over o = c mod 4 of |y[up g + o]|^2, o
 * ascending; oracle eo_om_group_partials) for tetra_etsi_timing_chunks (and _om).  D = M / 2 plan (up = 36) only. */
int tetra_channelize_om(tetra_ctx *ctx, const tetra_wb_plan *plan, const void *x, size_t Nw, void *y, size_t n_keep,
                        void *om);
/* Synthetic wideband capture: M carriers of tetra_synth_etsi bursts at fs/D, filter-bank
 * synthesised to fs, plus AWGN at per-carrier Es/N0 = snr_db.  Outputs as tetra_synth_etsi with
 * C = M and N = Nw / D + 1 (carrier k at +k fs / M, i.e. FFT bin k). */
int tetra_synth_wideband(tetra_ctx *ctx, const tetra_wb_plan *plan, size_t Nw, uint64_t seed, float snr_db,
                         float cfo_max, void *x, uint32_t *cell_init, int32_t *kinds, uint8_t *payload, double *t0);

/* ---------------------------------------------------------------- waterfall spectrum (C3)
 * Live spectrum / waterfall rows: frame f of channel c is x[c][f*hop .. f*hop + nfft), Hann
 * window (numpy.hanning), forward FFT, fftshift, power = 20 log10(|X| / nfft + 1e-20) in dBFS --
 * the display of /root/reference/tetraear/ui/modern.py:1928-1941 (one frame x[:2048] per chunk),
 * batched over channels and frames.  iq [C][N] in TETRA_CF32 / TETRA_SC16 / TETRA_CF64; out
 * [C][nframes][nfft] float32.  nfft = 2048 (the reference's fixed size); needs
 * (nframes - 1) * hop + nfft <= N.  Single-pass fused kernel (window + LDS FFT + dB). */
int tetra_waterfall(tetra_ctx *ctx, const void *iq, int iq_fmt, size_t C, size_t N, size_t nfft, size_t hop,
                    size_t nframes, float *out);

/* ---------------------------------------------------------------- FFT resampler
 * SignalProcessor.resample (/root/reference/tetraear/signal/processor.py:35-49 =
 * scipy.signal.resample(x, num)): x [C][Nx] complex (TETRA_CF32 or TETRA_CF64) -> y [C][num] in the
 * same precision; forward rocFFT, spectrum truncation / zero-padding with scipy's Nyquist
 * split/join, inverse rocFFT, scale num/Nx folded in. */
int tetra_resample(tetra_ctx *ctx, const void *x, int fmt, size_t C, size_t Nx, size_t num, void *y);

#ifdef __cplusplus
}
#endif
#endif /* TETRA_HIP_H */
