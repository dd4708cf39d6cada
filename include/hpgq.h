/*
 * hpgq.h — C-ABI of the MI355X FASTQ QC engine (libhpgq.so).
 *
 * This is the drop-in boundary for the per-read hot path of hpg-fastq
 * (SURVEY.md §8b).  Every entry point replaces one bioinfo-libs call made by
 * the reference's workflow workers, or the serial consumer merge that follows
 * them:
 *
 *   fastq_filter(reads, passed, failed, opts)     src/stats_fastq.c:224,
 *                                                 src/filter_fastq.c:148,
 *                                                 src/edit_fastq.c:166
 *   fastq_reads_stats(reads, rs_opts, fq_stats)   src/stats_fastq.c:230,244
 *   fastq_stats_consumer per-read + per-base merge src/stats_fastq.c:257-417
 *   fastq_edit(reads, opts)                       src/edit_fastq.c:154
 *   chaos_game_fill_tables(cg_data, batch, mode)  old/chaos_game.c:165-267
 *
 * The batch layout mirrors the SoA `fastq_batch_t` the old GPU path used
 * (fields evidenced at old/chaos_game.c:174-193): concatenated `seq` and
 * `quality` byte buffers plus `data_indices` with read i occupying
 * [data_indices[i], data_indices[i+1]).
 *
 * All functions return 0 on success or a negative HPGQ_E* code; no function
 * exits the process (the reference calls exit()/LOG_FATAL instead).
 * Plain pointers and sizes only — no C++ or framework types cross this line.
 */
#ifndef HPGQ_H
#define HPGQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------- */
/* constants                                                              */
/* ---------------------------------------------------------------------- */

/* src/commons_fastq.h:21-23 */
#define HPGQ_NO_VALUE   (-1)
#define HPGQ_MIN_VALUE  0
#define HPGQ_MAX_VALUE  100000

/* quality encodings (stats/edit --quality-encoding, src/stats_options.c:124-137) */
#define HPGQ_PHRED33 33
#define HPGQ_PHRED64 64

/* largest lmax: the dense per-position counters a ctx keeps on chip.
 * Reads of ANY length are merged: positions >= lmax of a longer read go to the
 * ctx's long-read tail (hpgq_read_counters_ext), like the reference's khash
 * maps, which have no length cap (src/stats_fastq.c:289-382). */
#define HPGQ_LMAX_LIMIT 1024
/* longest edit window (edit_left_length / edit_right_length): trims are
 * returned as two 16-bit fields (trim_out, hpgq_run_device) */
#define HPGQ_MAX_EDIT_LENGTH 65535
/* Device sequence / quality buffers must stay readable for this many bytes
 * past their last read (seq + data_indices[num_reads]): the engine fetches
 * unaligned 8-byte windows.  The bytes are never used. */
#define HPGQ_DEVICE_SLACK 8

/* error codes */
#define HPGQ_OK                  0
#define HPGQ_E_INVALID         (-1)   /* bad argument / parameter            */
#define HPGQ_E_HIP             (-2)   /* HIP runtime error                    */
#define HPGQ_E_NOMEM           (-3)   /* device or host allocation failed     */
#define HPGQ_E_READ_TOO_LONG   (-4)   /* not returned since round 6: reads of any
                                         length merge (kept for the ABI)        */
#define HPGQ_E_NO_DEVICE       (-5)   /* no HIP device                        */
#define HPGQ_E_RCCL            (-6)   /* RCCL communicator / collective error */
#define HPGQ_E_STATE           (-7)   /* call not valid in this ctx state     */
#define HPGQ_E_FORMAT          (-8)   /* malformed FASTQ text                 */
#define HPGQ_E_IO              (-9)   /* file open / read / write failed      */

/* ---------------------------------------------------------------------- */
/* batch                                                                  */
/* ---------------------------------------------------------------------- */

/*
 * SoA read batch (fastq_batch_t, old/chaos_game.c:176-193).  Read i is
 * seq[data_indices[i] .. data_indices[i+1]) and the same range of quality.
 * data_indices has num_reads+1 entries, is non-decreasing and is `int` like
 * the reference's, so one batch holds < 2 GiB of bases.  Offsets are
 * absolute into seq/quality (data_indices[0] need not be 0).
 */
typedef struct hpgq_batch {
  int64_t        num_reads;
  const char    *seq;
  const char    *quality;
  const int32_t *data_indices;
} hpgq_batch_t;

/* ---------------------------------------------------------------------- */
/* parameters                                                             */
/* ---------------------------------------------------------------------- */

/*
 * Engine parameters.  Filter fields follow fastq_filter_options_new's
 * argument order (src/filter_fastq.c:140-145); edit fields follow
 * fastq_edit_options_new (src/edit_fastq.c:148-151).  Values are already
 * defaulted the way the reference drivers do it (NO_VALUE -> MIN/MAX_VALUE,
 * src/filter_fastq.c:195-206); hpgq_params_init() gives those defaults.
 * Quality thresholds are Phred scores; the engine compares them with
 * (quality_char - phred).
 */
typedef struct hpgq_params {
  int32_t phred;              /* 33 or 64                                    */
  int32_t lmax;               /* dense per-position length, 1..HPGQ_LMAX_LIMIT
                                 (longer reads: the long-read tail)          */

  int32_t stats_on;           /* accumulate stats counters                   */
  int32_t filter_on;          /* apply the filter (else every read passes)   */
  int32_t edit_on;            /* 5'/3' trim before filter and stats          */
  int32_t paired;             /* batches are mate pairs; pair passes iff both */

  /* fastq_filter_options_new(...) */
  int32_t min_read_length, max_read_length;
  int32_t min_read_quality, max_read_quality;
  int32_t max_out_of_quality;
  int32_t left_length, min_left_quality, max_left_quality;
  int32_t right_length, min_right_quality, max_right_quality;
  int32_t max_N;

  /* fastq_edit_options_new(left_len, minL, maxL, right_len, minR, maxR, 0,0,0);
   * the lengths are at most HPGQ_MAX_EDIT_LENGTH (hpgq_open: HPGQ_E_INVALID) */
  int32_t edit_left_length, edit_min_left_quality, edit_max_left_quality;
  int32_t edit_right_length, edit_min_right_quality, edit_max_right_quality;
} hpgq_params_t;

/* Defaults: phred33, lmax 256, stats on, filter/edit off, ranges open. */
void hpgq_params_init(hpgq_params_t *p);

/* ---------------------------------------------------------------------- */
/* packed counters (what the stats consumer merges; RCCL all-reduces)     */
/* ---------------------------------------------------------------------- */

/*
 * One counter set is a flat uint64_t array.  Offsets depend on lmax:
 *
 *   [0 .. 8)                 scalars, HPGQ_S_*
 *   hist_len   [lmax+1]      reads per length               (kh_length_histogram)
 *   hist_meanq [256]         reads per round(mean raw Q)     (kh_quality_histogram)
 *   hist_gc    [101]         reads per 100*(G+C)/len         (kh_gc_histogram)
 *   pos_qsum   [lmax]        sum of raw quality per position (kh_acc_quality_per_nt)
 *   pos_base   [5][lmax]     A, C, G, T, N per position      (kh_num_*_per_nt)
 *
 * kh_count_quality_per_nt[j] = sum_{L>j} hist_len[L] and the scalar totals of
 * stats_counters_t (src/stats_fastq.h:35-73) are derived from these by
 * hpgq_counters_summary().  A paired ctx holds two sets back to back
 * (mate 1, mate 2).  Everything is an exact integer sum, so shards merge by
 * plain addition.
 *
 * Reads longer than lmax.  The reference merges every position of every read
 * (src/stats_fastq.c:338-382, khash keyed by j < read_length).  A merged read
 * of length L > lmax adds its positions < lmax, its mean-quality and GC bins
 * and every scalar to the set above (hpgq_read_counters) and counts in
 * HPGQ_S_LONG_READS; its positions >= lmax and its length go to the ctx's
 * long-read tail.  hpgq_read_counters_ext returns both as ONE set in the
 * layout above for lmax_ext = max(lmax, longest merged read) -- the set an
 * lmax of lmax_ext would have held (HPGQ_S_LONG_READS 0).
 */
#define HPGQ_S_NUM_INPUT      0  /* reads seen                                 */
#define HPGQ_S_NUM_PASSED     1  /* reads that passed (== input if no filter)  */
#define HPGQ_S_NUM_FAILED     2
#define HPGQ_S_NUM_EDITED     3  /* reads whose trim removed >= 1 base         */
#define HPGQ_S_NUM_STATS      4  /* reads merged into stats (counters->num_reads) */
#define HPGQ_S_ACC_MEANQ_FX16 5  /* sum of floor(65536*sumQraw/len) (acc_quality) */
#define HPGQ_S_LONG_READS     6  /* merged reads longer than lmax: their positions
                                    >= lmax and length are in the long-read tail
                                    (0 in an extended set)                    */
#define HPGQ_S_RESERVED       7
#define HPGQ_NUM_SCALARS      8

#define HPGQ_MEANQ_BINS 256
#define HPGQ_GC_BINS    101

static inline size_t hpgq_off_hist_len(int lmax)   { (void)lmax; return HPGQ_NUM_SCALARS; }
static inline size_t hpgq_off_hist_meanq(int lmax) { return HPGQ_NUM_SCALARS + (size_t)lmax + 1; }
static inline size_t hpgq_off_hist_gc(int lmax)    { return hpgq_off_hist_meanq(lmax) + HPGQ_MEANQ_BINS; }
static inline size_t hpgq_off_pos_qsum(int lmax)   { return hpgq_off_hist_gc(lmax) + HPGQ_GC_BINS; }
static inline size_t hpgq_off_pos_base(int lmax, int b) {
  return hpgq_off_pos_qsum(lmax) + (size_t)lmax * (size_t)(1 + b);
}
static inline size_t hpgq_counters_len(int lmax)   { return hpgq_off_pos_base(lmax, 5); }

/* base order inside pos_base */
#define HPGQ_BASE_A 0
#define HPGQ_BASE_C 1
#define HPGQ_BASE_G 2
#define HPGQ_BASE_T 3
#define HPGQ_BASE_N 4

/* Derived view of one counter set (stats_counters_t, src/stats_fastq.h:35-73). */
typedef struct hpgq_summary {
  uint64_t num_reads;        /* reads merged into stats                       */
  uint64_t num_passed, num_failed, num_edited, num_input;
  int32_t  min_length, max_length;   /* 100000 / 0 when no reads (stats_counters_new) */
  uint64_t acc_length;
  double   mean_length;
  double   mean_quality_raw; /* acc_quality/num_reads, raw units (fx16 exact sum) */
  uint64_t num_A, num_C, num_G, num_T, num_N;
} hpgq_summary_t;

int hpgq_counters_summary(const uint64_t *set, int lmax, hpgq_summary_t *out);

/* ---------------------------------------------------------------------- */
/* engine context                                                         */
/* ---------------------------------------------------------------------- */

typedef struct hpgq_ctx hpgq_ctx_t;

/* Open a ctx on HIP device `device` (its own stream, counters zeroed). */
int  hpgq_open(hpgq_ctx_t **ctx, int device, const hpgq_params_t *p);
void hpgq_close(hpgq_ctx_t *ctx);

/*
 * Resident path: all pointers are DEVICE pointers (HBM).  Runs the fused
 * edit -> filter -> stats kernel asynchronously on the ctx stream and
 * accumulates into the ctx counters.  mask_out[i] = 1 if read (pair) i
 * passed, 0 otherwise; trim_out[i] = trim_start | trim_end << 16 when edit
 * is on (for pairs: mate 1 in trim_out[i], mate 2 in trim_out[num_reads+i]).
 * Either output may be NULL.  For paired ctxs b2 is mate 2 (same num_reads),
 * else it must be NULL.  seq / quality must be readable HPGQ_DEVICE_SLACK bytes
 * past the data end (hpgq_run_host pads its own staging copy).
 */
int  hpgq_run_device(hpgq_ctx_t *ctx, const hpgq_batch_t *b, const hpgq_batch_t *b2,
                     uint8_t *mask_out, uint32_t *trim_out);

/*
 * Host path: pointers are HOST memory (any: malloc'd is fine).  The batch is
 * copied into one of the ctx's two page-locked staging slots (1 MB pieces,
 * each piece's H2D queued as soon as it is copied) and the call returns once
 * the caller's buffers have been read: they are reusable on return.  The
 * copies run on a second stream, so this batch's H2D overlaps the previous
 * batch's kernels.  mask_out / trim_out are filled by hpgq_sync() or
 * hpgq_read_counters() (or when the slot is reused two calls later), not
 * before: synchronising hpgq_stream() yourself does not fill them, and the
 * arrays must stay allocated until one of those calls.  hpgq_close() drops
 * the outputs of calls not delivered by then (it never writes them).
 * A stats-only caller passes NULL for both and needs no hpgq_sync per batch.
 */
int  hpgq_run_host(hpgq_ctx_t *ctx, const hpgq_batch_t *b, const hpgq_batch_t *b2,
                   uint8_t *mask_out, uint32_t *trim_out);

/*
 * Host path without the staging copy: reserve the ctx's next page-locked
 * staging slot for a batch of num_reads reads holding nbytes sequence bytes
 * (and as many quality bytes; nbytes2 for mate 2 of a paired ctx, else 0 and
 * b2 NULL).  On return b (b2) point into the slot: the caller writes
 * data_indices[0..num_reads] (starting at 0, ending at <= nbytes), the
 * sequence and the quality bytes there -- e.g. while packing its reads -- and
 * calls hpgq_run_host with exactly that batch, which then only queues the DMA
 * (no host copy; the reference worker's pack becomes the only one).  The
 * pointers are valid until that hpgq_run_host, or the next hpgq_host_batch /
 * hpgq_run_host on the ctx (which abandons the reservation); waiting for the
 * slot's previous batch, as hpgq_run_host does, may deliver that batch's
 * outputs.  Replaces the worker's malloc of the SoA batch
 * (fastq_stats_worker; src/stats_fastq.c:202-250).
 */
int  hpgq_host_batch(hpgq_ctx_t *ctx, int64_t num_reads, size_t nbytes, size_t nbytes2,
                     hpgq_batch_t *b, hpgq_batch_t *b2);

/* Wait for all work on the ctx stream (and deliver hpgq_run_host outputs).
 * Reads of any length are filtered, trimmed and merged.  The long-read tail
 * grows on the host: hpgq_run_host sizes it from the batch's own offsets before
 * the launch; hpgq_run_device cannot see them, so a device batch holding a
 * merged read longer than lmax + the tail reserved so far has that read's
 * excess positions merged HERE, by a second pass over the batch -- such a
 * device batch must stay valid until the next hpgq_sync / hpgq_read_counters /
 * hpgq_read_counters_ext / hpgq_reset (hpgq_reserve_length avoids the second
 * pass).  Never HPGQ_E_READ_TOO_LONG. */
int  hpgq_sync(hpgq_ctx_t *ctx);

/* Reserve the long-read tail for merged reads up to max_len bases (no-op when
 * max_len <= lmax or already reserved; waits for the ctx stream when it
 * grows the tail).  The CLI calls it with each parse unit's longest record
 * (hpgq_parser_max_length). */
int  hpgq_reserve_length(hpgq_ctx_t *ctx, int64_t max_len);

/* The counters of every merged read at full length: nm sets in the layout of
 * hpgq_counters_len(*lmax_ext), lmax_ext = max(lmax, longest merged read)
 * (HPGQ_S_LONG_READS 0; every other entry as an lmax of lmax_ext would give).
 * out == NULL: only *lmax_ext (size query).  Synchronises like
 * hpgq_read_counters.  After hpgq_allreduce the sum over the ranks, and then it
 * is COLLECTIVE: every rank of the communicator calls it (the ranks agree on
 * lmax_ext and sum their tails with two RCCL all-reduces). */
int  hpgq_read_counters_ext(hpgq_ctx_t *ctx, uint64_t *out, size_t n, int32_t *lmax_ext);

/* Zero the ctx counters (async on the ctx stream). */
int  hpgq_reset(hpgq_ctx_t *ctx);

/* Number of uint64 in this ctx's counter buffer (1 or 2 sets). */
size_t hpgq_counters_size(const hpgq_ctx_t *ctx);

/* Copy the counters to host memory (synchronises the ctx; like hpgq_sync it
 * also delivers pending hpgq_run_host masks / trims). */
int  hpgq_read_counters(hpgq_ctx_t *ctx, uint64_t *out, size_t n);

/* DEPRECATED no-op, kept only so that round-1 callers still link: the kernels
 * add their workgroup partials into the counters themselves (global
 * atomics), so the counter buffer holds the totals as soon as the ctx stream
 * has run the batch.  New code does not call it. */
int  hpgq_fold(hpgq_ctx_t *ctx);

/* Device pointer of this ctx's own counter buffer (for an external
 * all-reduce); holds the totals once the ctx stream has run the batches. */
uint64_t *hpgq_counters_device(hpgq_ctx_t *ctx);

/* HIP stream (hipStream_t) the ctx runs on.  Synchronising it waits for the
 * kernels but does not deliver hpgq_run_host outputs (hpgq_sync does). */
void *hpgq_stream(hpgq_ctx_t *ctx);

/* ---------------------------------------------------------------------- */
/* multi-GPU: RCCL over xGMI (one process per GPU)                        */
/* ---------------------------------------------------------------------- */

#define HPGQ_COMM_ID_BYTES 128

/* rank 0 creates the id and ships it to the other ranks out of band */
int  hpgq_comm_unique_id(char id[HPGQ_COMM_ID_BYTES]);
int  hpgq_comm_init(hpgq_ctx_t *ctx, int nranks, int rank, const char id[HPGQ_COMM_ID_BYTES]);
/* ncclAllReduce(sum, uint64) of the packed counters on the ctx stream, OUT OF
 * PLACE: the ctx keeps accumulating its own reads, the sum over the ranks goes
 * to a second buffer that hpgq_read_counters returns until the next run or
 * reset (so calling it twice, or after more batches, never double-counts). */
int  hpgq_allreduce(hpgq_ctx_t *ctx);
/* device pointer of the all-reduced counters */
uint64_t *hpgq_global_counters_device(hpgq_ctx_t *ctx);
/* ranks in the ctx's communicator (ncclCommCount); HPGQ_E_STATE without one.
 * The multi-GPU bench reports it next to its own world size
 * (the old tool's --gpu-num-devices, old/main_hpg_fastq_old.c:113,161). */
int  hpgq_comm_count(hpgq_ctx_t *ctx, int *count);

/*
 * Kernel routing for tests and A/B measurements only.  The
 * library never reads routing choices from the environment: a ctx runs the
 * automatic chain unless this is called.  It waits for the ctx stream and
 * re-plans the chain; counters are kept.
 *   AUTO        segmented kernel first (hex, or wide for lmax 157..252),
 *               adaptive hex/wide first stage, catch-all for the rest
 *   CATCH_ALL   the one-read-per-wave catch-all kernel alone
 *   FIRST_TRI / FIRST_HEX / FIRST_WIDE   that geometry first (not adaptive)
 * | NO_ADAPTIVE  (with AUTO) keep the first choice for every call
 */
#define HPGQ_ROUTE_AUTO        0
#define HPGQ_ROUTE_CATCH_ALL   1
#define HPGQ_ROUTE_FIRST_TRI   2
#define HPGQ_ROUTE_FIRST_HEX   3
#define HPGQ_ROUTE_FIRST_WIDE  4
#define HPGQ_ROUTE_NO_ADAPTIVE 0x10
int  hpgq_debug_set_route(hpgq_ctx_t *ctx, int route);

/* ---------------------------------------------------------------------- */
/* chaos-game (CGR) accumulator, old/chaos_game.c:165-267                 */
/* ---------------------------------------------------------------------- */

#define HPGQ_CGR_ALL_READS        0
#define HPGQ_CGR_ONLY_VALID_READS 1   /* mode == ONLY_VALID_READS (:188) */

typedef struct hpgq_cgr hpgq_cgr_t;

/*
 * k: word size (dim = 2^k, tables dim x dim, 1 <= k <= 12);
 * base_quality: subtracted k times per word (chaos_game_data_init :97).
 */
int  hpgq_cgr_open(hpgq_cgr_t **cg, int device, int k, int base_quality);
void hpgq_cgr_close(hpgq_cgr_t *cg);

/*
 * One chaos_game_fill_tables() call over a DEVICE batch.  The double CGR
 * state starts at (dim/2, dim/2) for every call and is carried across the
 * reads of the batch exactly as the reference does.  status (device, may be
 * NULL) is read_status[]; in ONLY_VALID_READS mode reads with status[i] != 1
 * (VALID_READ) are skipped.
 */
int  hpgq_cgr_fill_device(hpgq_cgr_t *cg, const hpgq_batch_t *b, const uint8_t *status, int mode);
int  hpgq_cgr_sync(hpgq_cgr_t *cg);
int  hpgq_cgr_reset(hpgq_cgr_t *cg);
/* table_seq, table_q: dim*dim uint32 each, row-major [co_x][co_y]; word_count: fq_word_count */
int  hpgq_cgr_read(hpgq_cgr_t *cg, uint32_t *table_seq, uint32_t *table_q, uint32_t *word_count);
void *hpgq_cgr_stream(hpgq_cgr_t *cg);
/* reads the last fill call had to replay sequentially (diagnostic) */
int64_t hpgq_cgr_last_replays(hpgq_cgr_t *cg);

/*
 * Multi-GPU (read-sharded fills, one process per GPU): RCCL communicator
 * from a unique id (hpgq_comm_unique_id), then one all-reduce of
 * [table_seq | table_q | word_count] as uint32 sums, which wrap like the
 * reference's unsigned tables (old/chaos_game.c:253-258).  Out of place:
 * hpgq_cgr_read returns the sums until the next fill or reset.
 */
int  hpgq_cgr_comm_init(hpgq_cgr_t *cg, int nranks, int rank, const char id[HPGQ_COMM_ID_BYTES]);
int  hpgq_cgr_allreduce(hpgq_cgr_t *cg);
/* ranks in the chaos-game communicator (ncclCommCount); HPGQ_E_STATE without one */
int  hpgq_cgr_comm_count(hpgq_cgr_t *cg, int *count);
/* device pointer of the all-reduced [table_seq | table_q | word_count] */
uint32_t *hpgq_cgr_global_device(hpgq_cgr_t *cg);

/*
 * Path selection.  AUTO (default): for k <= 7 (either mode) a coalesced
 * integer pass computes each word's cell from its own k bases, which is
 * provably the reference's (int)f cell unless some axis sees a run of
 * >= 48-k toward-dim moves or a counted read holds bytes other than A/C/G/T/N
 * or qualities >= 128; such a call is redone by the exact double simulation
 * on the device.  In ONLY_VALID_READS mode the skipped reads' bytes count as
 * absent (they move nothing, :188).  EXACT: always the exact simulation.
 * Both are bit-identical to old/chaos_game.c:165-267.
 */
#define HPGQ_CGR_PATH_AUTO  0
#define HPGQ_CGR_PATH_EXACT 1
int  hpgq_cgr_set_path(hpgq_cgr_t *cg, int path);
/* 1 if a fill since the previous sync ran the exact simulation, 0 if the
 * stream pass sufficed for all of them (read after hpgq_cgr_sync).  A
 * streamed fill whose gate is set is simulated exactly inside the next
 * hpgq_cgr_sync / hpgq_cgr_read / hpgq_cgr_reset, so its batch must stay
 * valid until then (as for any asynchronous fill). */
int  hpgq_cgr_last_exact(hpgq_cgr_t *cg);

/*
 * CGR post-processing on the host (O(4^k), old/chaos_game.c:269-593); tables
 * are row-major [co_x][co_y] of dim*dim cells as hpgq_cgr_read returns them.
 *   genomic-signature (GS) file = header_gs_t (old/chaos_game.h:65-70: char
 *   gs_filename[180], u32 word_size_k, dim_x, dim_y, ref_word_count) + the
 *   dim*dim u32 table.
 */
#define HPGQ_GS_HEADER_BYTES 196
/* chaos_game_load_table_gs_direct (:297-318) */
int  hpgq_cgr_load_gs(const char *path, int k, uint32_t *table_gs, uint32_t *ref_word_count);
/* header_gs_init (:43-50) + the table: writes a GS file for a reference */
int  hpgq_cgr_write_gs(const char *path, int k, const uint32_t *table, uint32_t word_count);
/* chaos_game_calculate_table_dif (:320-373): int table_dif = seq*128/(fq/4^k) - gs*128/(ref/4^k) */
int  hpgq_cgr_table_dif(int k, const uint32_t *table_seq, uint32_t fq_word_count,
                        const uint32_t *table_gs, uint32_t ref_word_count, int32_t *table_dif,
                        int32_t *highest, int32_t *lowest);
/* chaos_game_validate_table_dif (:375-408): mean and standard deviation of table_dif */
int  hpgq_cgr_dif_stats(int k, const int32_t *table_dif, double *mean, double *std_dev);
/* chaos_game_normalize_quality_table_ (:487-502), in place */
int  hpgq_cgr_normalize_quality(int k, const uint32_t *table_seq, uint32_t *table_q);
/* chaos_game_generate_pgm_file_ (:521-593) */
int  hpgq_cgr_write_pgm(const char *path, int k, const uint32_t *table, double norm);
/* chaos_game_write_table_images (:410-472): <dir>/<fq file>_k=<k>_FG.pgm, _QQ.pgm
 * (normalises table_q in place) and, when table_dif is given, _FG_dif.pgm */
int  hpgq_cgr_write_images(const char *report_dir, const char *fq_path, int k,
                           const uint32_t *table_seq, uint32_t *table_q, uint32_t fq_word_count,
                           const int32_t *table_dif);

/* ---------------------------------------------------------------------- */
/* stats --kmers: 5-mer counts (src/stats_options.c:274, merge              */
/* src/stats_fastq.c:384-410, report src/stats_report.c:492-563)            */
/* ---------------------------------------------------------------------- */

#define HPGQ_KMER_K    5
#define HPGQ_NUM_KMERS 1024   /* NUM_KMERS, src/stats_fastq.h:58 */

/*
 * Build-defined (the per-read k-mer code is in the absent bioinfo-libs;
 * DESIGN.md §2.5): 5-mers of exact uppercase A/C/G/T, id = sum code_i *
 * 4^(4-i) with A=0 C=1 G=2 T=3, counted at every start position
 * p <= len-5 of every counted read.  by_pos is [HPGQ_NUM_KMERS][npos] u64
 * (counter_by_pos); a k-mer's counter is its row sum.  hpgq_kmers_read gives
 * the dense starts p < npos = lmax-4; starts >= npos of longer reads (the
 * reference's counter_by_pos grows with the read, src/stats_fastq.c:394-407)
 * are in the tail, and hpgq_kmers_read_ext returns all of them as
 * [HPGQ_NUM_KMERS][npos_ext], npos_ext = max(lmax, longest counted read) - 4.
 * The tail's reservation and second pass work as the engine's (hpgq_sync).
 */
typedef struct hpgq_kmers hpgq_kmers_t;

/* stream: run on this HIP stream (e.g. hpgq_stream(ctx), so counting sees the
 * engine's mask of the same batch), or NULL for an own stream */
int  hpgq_kmers_open(hpgq_kmers_t **km, int device, int lmax, void *stream);
void hpgq_kmers_close(hpgq_kmers_t *km);
/* Count a DEVICE batch, async; mask (device, may be NULL): only reads with
 * mask[i] == 1 (the engine's mask_out: passed) are counted. */
int  hpgq_kmers_count_device(hpgq_kmers_t *km, const hpgq_batch_t *b, const uint8_t *mask);
int  hpgq_kmers_sync(hpgq_kmers_t *km);
int  hpgq_kmers_reset(hpgq_kmers_t *km);
/* HPGQ_NUM_KMERS * (lmax-4) (0 when lmax < 5) */
size_t hpgq_kmers_size(const hpgq_kmers_t *km);
/* copy by_pos to host (synchronises); n >= hpgq_kmers_size() */
int  hpgq_kmers_read(hpgq_kmers_t *km, uint64_t *by_pos, size_t n);
/* device pointer of by_pos (for an external all-reduce) */
uint64_t *hpgq_kmers_device(hpgq_kmers_t *km);
/* tail for counted reads up to max_len bases (cf. hpgq_reserve_length) */
int  hpgq_kmers_reserve_length(hpgq_kmers_t *km, int64_t max_len);
/* every start: [HPGQ_NUM_KMERS][*npos_ext] (by_pos == NULL: size query) */
int  hpgq_kmers_read_ext(hpgq_kmers_t *km, uint64_t *by_pos, size_t n, int32_t *npos_ext);

/* ---------------------------------------------------------------------- */
/* FASTQ text -> device batch (the parsing half of the producer's          */
/* fastq_fread_se, src/stats_fastq.c:183, moved onto the GPU)              */
/* ---------------------------------------------------------------------- */

/*
 * Records are 4 lines: "@header", sequence, "+[header]", quality (as long as
 * the sequence); "\n" or "\r\n" line ends.  A parse unit is whole records,
 * the last one ending in a newline.
 */
typedef struct hpgq_parser hpgq_parser_t;

/* Bytes of buf[0, n) that form whole records; the rest starts the next unit.
 * at_eof: the data ends at n (returns n; the caller appends a final newline
 * when the file lacks one).  0: no complete record yet.  Host-only. */
int64_t hpgq_fastq_complete_prefix(const char *buf, int64_t n, int at_eof);

/* stream: the stream to parse on (e.g. hpgq_stream(ctx), so the engine runs
 * after it), or NULL for a stream of its own */
int  hpgq_parser_open(hpgq_parser_t **ps, int device, void *stream);
void hpgq_parser_close(hpgq_parser_t *ps);
/* Parse text[0, n) (n < 2^31) into a device batch owned by the parser, valid
 * until its next parse; `out` gets device pointers and num_reads.  _host
 * copies the text to the device first.  HPGQ_E_FORMAT on malformed records. */
int  hpgq_parse_host(hpgq_parser_t *ps, const char *text, int64_t n, hpgq_batch_t *out);
int  hpgq_parse_device(hpgq_parser_t *ps, const char *text_dev, int64_t n, hpgq_batch_t *out);
/* offsets into the last parsed text, num_reads u32 each (any may be NULL):
 * record start ('@'), sequence, '+' line, quality */
int  hpgq_parse_records(hpgq_parser_t *ps, uint32_t *rec_start, uint32_t *seq_start,
                        uint32_t *plus_start, uint32_t *qual_start);
void *hpgq_parser_stream(hpgq_parser_t *ps);
/* the longest record of the last parse (0 when empty): the engine's and the
 * k-mer counter's hpgq_*reserve_length before they run the batch */
int64_t hpgq_parser_max_length(hpgq_parser_t *ps);

/* ---------------------------------------------------------------------- */
/* synthetic input (bench / tests): counter-based, identical on host & GPU */
/* ---------------------------------------------------------------------- */

typedef struct hpgq_synth {
  uint64_t seed;
  int32_t  read_length;      /* L                                            */
  int32_t  trunc_pct;        /* % of reads truncated to U[20, L]            */
  int32_t  bad_pct;          /* % of reads with Q centred at 12             */
  int32_t  n_per_1024;       /* 'N' probability x 1024                      */
  int32_t  phred;            /* quality offset                              */
  int32_t  mate;             /* 0 or 1 (mate 2 reuses mate 1's lengths)     */
} hpgq_synth_t;

/* read length of read `idx` (host, no device needed) */
int32_t hpgq_synth_length(const hpgq_synth_t *s, int64_t idx);
/* data_indices (n+1 entries, starting at 0) of reads [first, first+n) */
int  hpgq_synth_indices_host(const hpgq_synth_t *s, int64_t first, int64_t n, int32_t *idx_host);
/* Fill seq/quality of reads [first, first+n) on the device; idx_dev must
 * already hold hpgq_synth_indices_host()'s output. Async on `stream`. */
int  hpgq_synth_device(const hpgq_synth_t *s, int64_t first, int64_t n,
                       char *seq_dev, char *qual_dev, const int32_t *idx_dev, void *stream);

/* number of visible HIP devices (0 when none or the runtime fails) */
int  hpgq_device_count(void);
/* NUMA node of HIP device `device` (its PCI function's numa_node in sysfs),
 * -1 when unknown: host threads and buffers that feed it belong there */
int  hpgq_device_numa_node(int device);

const char *hpgq_strerror(int code);
const char *hpgq_version(void);
/* the first engine kernel instance of a ctx's chain (for profiles / bench
 * reports) and the whole chain ("first -> follow-up -> ..."); DESIGN.md §4.0 */
const char *hpgq_kernel_name(const hpgq_ctx_t *ctx);
const char *hpgq_kernel_chain(const hpgq_ctx_t *ctx);

/* memory helpers for HIP-free hosts (the C CLI): page-locked host buffers
 * (fast, asynchronous H2D), device buffers, and a device -> host copy queued
 * on a ctx stream (complete after hpgq_sync) */
int  hpgq_host_alloc(void **ptr, size_t bytes);
void hpgq_host_free(void *ptr);
int  hpgq_device_alloc(int device, void **ptr, size_t bytes);
void hpgq_device_free(void *ptr);
int  hpgq_copy_to_host(hpgq_ctx_t *ctx, void *dst, const void *src_dev, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* HPGQ_H */
