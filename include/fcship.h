/*
 * fcship.h — C-ABI of the MI355X (gfx950) hot-path library libfcship.so.
 *
 * This is the drop-in boundary for the two dynamic-programming hot paths that
 * the reference's `fcs-genome` CLI reaches only through external processes:
 *
 *   PairHMM forward algorithm (htc / mutect2)
 *     reference call-out : HTCWorker::setup builds `java -jar GATK HaplotypeCaller
 *                          ... --native-pair-hmm-threads=N`
 *                          (/root/reference/src/workers/HTCWorker.cpp:51-85),
 *                          Mutect2Worker::setup (/root/reference/src/workers/Mutect2Worker.cpp:109-192),
 *                          FPGA offload via the Blaze NAM daemon started by
 *                          BackgroundExecutor (/root/reference/src/worker-htc.cpp:100-112,
 *                          /root/reference/src/worker-mutect2.cpp:153-165).
 *     interface replaced : GKL IntelPairHmm.computeLikelihoodsNative(ReadDataHolder[],
 *                          HaplotypeDataHolder[], double[] likelihoods) [EXT, not
 *                          vendored]; see fcs_phmm_compute.
 *
 *   BWA-MEM banded Smith-Waterman (align)
 *     reference call-out : BWAWorker::setup builds `bwa-flow mem ... --offload
 *                          --use_fpga --fpga_path=<root>/fpga/sw.xclbin`
 *                          (/root/reference/src/workers/BWAWorker.cpp:134-166;
 *                          config keys /root/reference/src/config.cpp:297-300).
 *     interface replaced : bwa ksw.c ksw_extend2() / ksw_global2() [EXT, not
 *                          vendored]; see fcs_ksw_extend2 / fcs_ksw_global2 (same
 *                          argument lists) and the batched fcs_bsw_* entry points.
 *
 * Conventions:
 *   - every function returns FCS_OK (0) or a negative FCS_ERR_* code; the
 *     message of the last failure on the calling thread is fcs_last_error();
 *   - no C++ exceptions cross the boundary;
 *   - the caller owns every buffer; nothing is retained after a synchronous
 *     return;
 *   - entry points are thread-safe; each (thread, device) pair uses its own
 *     HIP stream for the synchronous host-pointer calls;
 *   - `device` selects the GPU (the Executor's GPU slot);
 *   - the *_dev entry points take DEVICE pointers and a hipStream_t (passed as
 *     void*), enqueue work and return without synchronising.  The library
 *     keeps side streams and events per launch stream it has seen (a stream
 *     costs ~3.5 ms to create): use long-lived launch streams, and call
 *     fcs_stream_release before destroying one.
 *
 * Nothing here falls back to the CPU: if no gfx950 device is present the
 * calls fail with FCS_ERR_DEVICE.
 */
#ifndef FCSHIP_H
#define FCSHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FCS_OK 0
#define FCS_ERR_INVALID (-1)     /* bad argument */
#define FCS_ERR_DEVICE (-2)      /* no device / HIP runtime failure */
#define FCS_ERR_NOMEM (-3)       /* allocation failure */
#define FCS_ERR_UNSUPPORTED (-4) /* outside the supported envelope (e.g. m != 5) */

/* ------------------------------------------------------------------ common */
int fcs_device_count(void);
const char* fcs_last_error(void);
const char* fcs_version(void);
/* Build/ABI self-description: number of symbols this library exports that are
 * declared in this header (used by the loader test). */
int fcs_abi_symbol_count(void);
/* Brings `device` up ahead of the first real call: the HIP runtime, the code
 * objects and the GKL tables (a 1x1 PairHMM call), and `sessions` pooled
 * call sessions (<= 0: the pool's size, FCS_SESSIONS_PER_DEVICE, default 4).
 * A session is the stream, side streams and staging arenas the host-pointer
 * entry points lease for one call; a call finding every session busy waits
 * for one.  fcs-genome runs this in the background while the first shards
 * decode their reads (the reference's BackgroundExecutor role,
 * /root/reference/include/fcs-genome/BackgroundExecutor.h:12). */
int fcs_device_warmup(int32_t device, int32_t sessions);
/* Drops the side streams, events and SW schedule workspace the library keeps
 * for launch stream `stream` on `device` (created at its first *_dev call).
 * Call it after the stream's work has finished and before destroying the
 * stream; a later *_dev call on the same stream recreates them. */
int fcs_stream_release(int32_t device, void* stream);
/* Releases everything the library holds on `device` (session streams, pinned
 * and device arenas, plans, tables) and resets the device, so the process's
 * GPU teardown happens now instead of after its last output: `fcs-genome`
 * calls it beside the VCF tail.  FCS_ERR_INVALID while a synchronous
 * (host-pointer) call on the device is still running; while the reset runs,
 * such calls on the device fail with FCS_ERR_INVALID (fcs_bgzf_inflate_try
 * answers FCS_BGZF_BUSY).  The *_dev entry points on caller streams and plans
 * the caller owns are not tracked: the caller finishes them first.  A later
 * call on the device sets everything up again.
 * The reset frees every allocation of the process on the device, other
 * libraries' included: call it only when nothing else holds device memory. */
int fcs_device_release(int32_t device);

/* ----------------------------------------------------------------- PairHMM */
/* One read: bases + the four per-base quality arrays GATK hands to the PairHMM
 * (base quality, insertion GOP, deletion GOP, gap-continuation penalty), all
 * already preprocessed by the caller exactly as for GKL (quals are used &127). */
typedef struct {
  const uint8_t* bases;
  const uint8_t* base_q;
  const uint8_t* ins_q;
  const uint8_t* del_q;
  const uint8_t* gcp;
  int32_t len;
} fcs_phmm_read;

typedef struct {
  const uint8_t* bases;
  int32_t len;
} fcs_phmm_hap;

typedef struct {
  int32_t device;           /* GPU ordinal */
  int32_t use_fp64_rescue;  /* 1: recompute pairs whose fp32 result < rescue_threshold in fp64 (GKL) */
  float rescue_threshold;   /* GKL MIN_ACCEPTED = 1e-28f */
  int32_t exact_order;      /* 1: no FMA contraction, GKL operation order (bitwise vs the fp32 oracle);
                               0: FMA-contracted fast path (default) */
} fcs_phmm_opts;

/* Defaults: device 0, rescue on, 1e-28f, fast path. */
void fcs_phmm_opts_default(fcs_phmm_opts* o);

/* Replacement for GKL computeLikelihoodsNative: every read against every
 * haplotype, log10 likelihoods written read-major:
 * out_log10[r * n_haps + h].  Host pointers, synchronous. */
int fcs_phmm_compute(const fcs_phmm_read* reads, int32_t n_reads, const fcs_phmm_hap* haps,
                     int32_t n_haps, double* out_log10, const fcs_phmm_opts* opts);

/* One active region: its reads x haplotypes matrix, written read-major to
 * out_log10[r * n_haps + h] (the per-region call GATK's
 * PairHMMLikelihoodCalculationEngine makes [EXT]). */
typedef struct {
  const fcs_phmm_read* reads;
  int32_t n_reads;
  const fcs_phmm_hap* haps;
  int32_t n_haps;
  double* out_log10;
} fcs_phmm_region;

/* Active-region batching: many regions in one device
 * pass, each region's result identical to fcs_phmm_compute on that region
 * alone.  Host pointers, synchronous. */
int fcs_phmm_compute_regions(const fcs_phmm_region* regions, int32_t n_regions, const fcs_phmm_opts* opts);

/* Flat structure-of-arrays pair batch.  Read k occupies
 * [read_off[k], read_off[k] + read_len[k]) of each of the five read byte
 * arrays; hap k occupies [hap_off[k], hap_off[k] + hap_len[k]) of hap_bases;
 * pair p is (pair_read[p], pair_hap[p]).  max_read_len / max_hap_len must bound
 * every length (they size on-chip buffers). */
typedef struct {
  const uint8_t* read_bases;
  const uint8_t* read_bq;
  const uint8_t* read_iq;
  const uint8_t* read_dq;
  const uint8_t* read_gcp;
  const int64_t* read_off;
  const int32_t* read_len;
  int64_t n_reads;
  const uint8_t* hap_bases;
  const int64_t* hap_off;
  const int32_t* hap_len;
  int64_t n_haps;
  const int32_t* pair_read;
  const int32_t* pair_hap;
  int64_t n_pairs;
  int64_t read_bytes; /* total bytes in each read byte array */
  int64_t hap_bytes;  /* total bytes in hap_bases */
  int32_t max_read_len;
  int32_t max_hap_len;
} fcs_phmm_batch;

/* Host-pointer batch (synchronous): out_log10[p] for every pair. */
int fcs_phmm_compute_pairs(const fcs_phmm_batch* b, double* out_log10, const fcs_phmm_opts* opts);

/* Device-resident path.  A plan owns the scratch (schedule, sort temp storage,
 * rescue list) for batches up to max_pairs pairs. */
typedef struct fcs_phmm_plan fcs_phmm_plan;
/* Multi-GPU static partition of one pair batch (the
 * reference's GPU/host placement is src/Executor.cpp:262): the pairs are cut
 * into n contiguous slices of ~equal total R*H cells (the cut where the
 * running cost first reaches k/n of the total; cuts[0..n], cuts[n] = n_pairs)
 * and each slice runs on its device from its own host thread, writing its
 * disjoint slice of out_log10.  No collective; results equal the one-device
 * call's.  fcs_phmm_last_rescued reports the sum over the slices. */
int fcs_phmm_partition(const fcs_phmm_batch* b, int32_t n_slices, int64_t* cuts);
int fcs_phmm_compute_pairs_multi(const fcs_phmm_batch* b, double* out_log10, const fcs_phmm_opts* opts,
                                 const int32_t* devices, int32_t n_devices);

int fcs_phmm_plan_create(int32_t device, int64_t max_pairs, fcs_phmm_plan** plan);
int fcs_phmm_plan_destroy(fcs_phmm_plan* plan);
/* Stage 1: order pairs into 4-pair wave groups by (read len, hap len). */
int fcs_phmm_dev_schedule(fcs_phmm_plan* plan, const fcs_phmm_batch* dev_batch, void* stream);
/* Stage 2: fp32 forward pass over the schedule; writes out_log10 for pairs
 * that pass the rescue threshold and queues the others. */
int fcs_phmm_dev_forward(fcs_phmm_plan* plan, const fcs_phmm_batch* dev_batch, double* dev_out_log10,
                         const fcs_phmm_opts* opts, void* stream);
/* Stage 3: fp64 rescue pass over the queued pairs (no-op if none). */
int fcs_phmm_dev_rescue(fcs_phmm_plan* plan, const fcs_phmm_batch* dev_batch, double* dev_out_log10,
                        const fcs_phmm_opts* opts, void* stream);
/* Stages 1-3 back to back. */
int fcs_phmm_dev_run(fcs_phmm_plan* plan, const fcs_phmm_batch* dev_batch, double* dev_out_log10,
                     const fcs_phmm_opts* opts, void* stream);
/* Number of pairs the last forward pass queued for rescue (synchronises the stream). */
int fcs_phmm_plan_rescue_count(fcs_phmm_plan* plan, void* stream, int64_t* count);
/* Pairs the fp64 rescue recomputed in the calling thread's last synchronous
 * fcs_phmm_compute / _regions / _pairs call (0 when rescue is off). */
int fcs_phmm_last_rescued(int64_t* count);
/* Device time of the calling thread's last synchronous PairHMM call, from HIP
 * events on its stream: schedule + fp32 forward + fp64 rescue, and the rescue
 * stage alone (ms).  Host staging and PCIe copies are not included. */
int fcs_phmm_last_device_ms(double* device_ms, double* rescue_ms);

/* -------------------------------------------------------------- banded SW */
typedef struct {
  int32_t qlen, tlen, h0, w;
  const uint8_t* query;  /* bases coded 0..4 (A,C,G,T,N) as in bwa */
  const uint8_t* target;
} fcs_bsw_task;

typedef struct {
  int8_t mat[25]; /* 5x5 scoring matrix, row = target base, col = query base */
  int32_t o_del, e_del, o_ins, e_ins, end_bonus, zdrop;
} fcs_bsw_params;

typedef struct {
  int32_t score, qle, tle, gtle, gscore, max_off;
} fcs_bsw_result;

/* bwa defaults: a=1, b=4 (N scores -1), o=6, e=1, end_bonus=5, zdrop=100. */
void fcs_bsw_params_default(fcs_bsw_params* p);

/* Batched ksw_extend2 (host pointers, synchronous). */
int fcs_bsw_extend(const fcs_bsw_task* tasks, int32_t n, const fcs_bsw_params* params,
                   fcs_bsw_result* results, int32_t device);
/* The same over several devices: contiguous slices of ~equal
 * qlen * tlen, one device and one host thread each, disjoint result slices. */
int fcs_bsw_extend_multi(const fcs_bsw_task* tasks, int32_t n, const fcs_bsw_params* params,
                         fcs_bsw_result* results, const int32_t* devices, int32_t n_devices);

/* Packed structure-of-arrays extension batch (device or host pointers
 * depending on the entry point).  Task k: query bytes
 * qbuf[qoff[k] .. +qlen[k]), target bytes tbuf[toff[k] .. +tlen[k]).
 * max_qlen / max_tlen must bound every qlen / tlen (they size on-chip and
 * scratch buffers). */
typedef struct {
  const uint8_t* qbuf;
  const int64_t* qoff;
  const int32_t* qlen;
  const uint8_t* tbuf;
  const int64_t* toff;
  const int32_t* tlen;
  const int32_t* h0;
  const int32_t* w;
  int64_t n;
  int64_t qbytes;
  int64_t tbytes;
  int32_t max_qlen;
  int32_t max_tlen;
} fcs_bsw_batch;

/* Device path: res = 6 int32 per task (score, qle, tle, gtle, gscore,
 * max_off); cells (nullable) = evaluated cells per task (int64). */
int fcs_bsw_extend_dev(const fcs_bsw_batch* dev_batch, const fcs_bsw_params* params, int32_t* dev_res,
                       int64_t* dev_cells, int32_t device, void* stream);

/* Reusable device scratch for fcs_bsw_extend_plan (schedule sort buffers for
 * batches of up to max_tasks tasks); fcs_bsw_extend_dev keeps the same scratch
 * per launch stream (grown with hipMalloc when a batch outgrows it, dropped by
 * fcs_stream_release).  No entry point uses the stream-ordered pool
 * (hipMallocAsync): on this runtime it hands memory live on one stream to
 * another (tools/micro/pin_reuse.hip). */
typedef struct fcs_bsw_plan fcs_bsw_plan;
int fcs_bsw_plan_create(int32_t device, int64_t max_tasks, fcs_bsw_plan** plan);
int fcs_bsw_plan_destroy(fcs_bsw_plan* plan);
int fcs_bsw_extend_plan(fcs_bsw_plan* plan, const fcs_bsw_batch* dev_batch, const fcs_bsw_params* params,
                        int32_t* dev_res, int64_t* dev_cells, void* stream);

/* Host-pointer packed batch (synchronous). */
int fcs_bsw_extend_batch(const fcs_bsw_batch* host_batch, const fcs_bsw_params* params, int32_t* res,
                         int64_t* cells, int32_t device);

/* Batched ksw_global2 (host pointers, synchronous).  Task k uses tasks[k].w as
 * the band and ignores h0.  scores[k] = global score; CIGAR ops of task k are
 * written to cigar_arena[cigar_off[k] .. cigar_off[k] + cigar_cap[k]) and the
 * true op count to n_cigar[k] (FCS_ERR_INVALID if any count exceeds its cap;
 * qlen + tlen always suffices). */
int fcs_bsw_global(const fcs_bsw_task* tasks, int32_t n, const fcs_bsw_params* params, int32_t* scores,
                   uint32_t* cigar_arena, const int64_t* cigar_off, const int32_t* cigar_cap,
                   int32_t* n_cigar, int32_t device);

/* Device path of ksw_global2 (stream-ordered, no host sync): task k of
 * dev_batch aligned with band dev_batch->w[k]; dev_scores[k] = global score.
 * Scores only when dev_cigar is null.  Otherwise dev_zbuf holds task k's
 * direction matrix at dev_zoff[k] (min(qlen, 2w+1) * tlen bytes, caller-sized;
 * zbytes = its total), the CIGAR ops go to dev_cigar[dev_cigar_off[k] ..
 * + dev_cigar_cap[k]) and their count to dev_n_cigar[k] (a count above the cap
 * means the ops were truncated). */
int fcs_bsw_global_dev(const fcs_bsw_batch* dev_batch, const fcs_bsw_params* params, int32_t* dev_scores,
                       uint8_t* dev_zbuf, int64_t zbytes, const int64_t* dev_zoff, uint32_t* dev_cigar,
                       const int64_t* dev_cigar_off, const int32_t* dev_cigar_cap, int32_t* dev_n_cigar,
                       int32_t device, void* stream);

/* Batched ksw_align2: bwa's local Smith-Waterman with the second-best score
 * and the alignment start (bwa ksw.c ksw_align2 = ksw_u8 / ksw_i16 + the
 * KSW_XSTART reverse pass), the kernel of bwa mem's mate rescue (mem_matesw:
 * xtra = KSW_XSUBO | KSW_XSTART | (l_ms * a < 250 ? KSW_XBYTE : 0) |
 * min_seed_len * a).  Replaces the call inside bwa-flow reached from
 * /root/reference/src/workers/BWAWorker.cpp:134-166.  Task k: query / target
 * codes 0..4 (qlen <= 1024), tasks[k].h0 / .w ignored, xtra[k] bwa's xtra word.
 * out[k] = bwa's kswr_t (score, te, qe, score2, te2, tb, qb; -1 where bwa
 * leaves -1). */
/* Task limits of fcs_bsw_align: longer queries or targets make the whole
 * call fail with FCS_ERR_UNSUPPORTED (callers filter them first). */
#define FCS_ALIGN_MAX_QLEN 1024
#define FCS_ALIGN_MAX_TLEN 54000
#define FCS_KSW_XBYTE 0x10000
#define FCS_KSW_XSTOP 0x20000
#define FCS_KSW_XSUBO 0x40000
#define FCS_KSW_XSTART 0x80000
typedef struct {
  int32_t score, te, qe, score2, te2, tb, qb;
} fcs_kswr;
int fcs_bsw_align(const fcs_bsw_task* tasks, int32_t n, const fcs_bsw_params* params, const int32_t* xtra,
                  fcs_kswr* out, int32_t device);
/* Device path (stream-ordered, no host sync): dev_xtra[k], dev_out[k] as above. */
int fcs_bsw_align_dev(const fcs_bsw_batch* dev_batch, const fcs_bsw_params* params, const int32_t* dev_xtra,
                      fcs_kswr* dev_out, int32_t device, void* stream);

/* Signature twins of bwa's ksw.c entry points, running on GPU `device` 0 (or
 * the device set by fcs_set_default_device).  m must be 5.  They return the
 * score exactly as bwa does; because a global score can be negative, failure
 * is signalled by FCS_KSW_FAILED (INT32_MIN) plus fcs_last_error().
 * fcs_ksw_global2 returns the CIGAR in *cigar allocated with malloc(), as bwa
 * does (caller frees). */
#define FCS_KSW_FAILED (-2147483647 - 1)
int fcs_ksw_extend2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m,
                    const int8_t* mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                    int end_bonus, int zdrop, int h0, int* qle, int* tle, int* gtle, int* gscore,
                    int* max_off);
int fcs_ksw_global2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m,
                    const int8_t* mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                    int* n_cigar, uint32_t** cigar);
/* bwa's kswr_t ksw_align2(qlen, query, tlen, target, m, mat, o_del, e_del,
 * o_ins, e_ins, xtra, qry); qry must be NULL (no cached profile).  On failure
 * the returned score is FCS_KSW_FAILED (fcs_last_error()). */
fcs_kswr fcs_ksw_align2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                        int o_del, int e_del, int o_ins, int e_ins, int xtra, void** qry);
int fcs_set_default_device(int32_t device);

/* ------------------------------------------------------ BGZF inflate (§8 f3) */
/* The BAM / BGZF container in front of the PairHMM path:
 * the reference's `htc` reads its window through htslib's bgzf_read
 * (htslib bgzf.c inflate_block: one raw-DEFLATE member at a time, CRC-32
 * checked); these entry points inflate a run of whole members on the GPU.
 *
 * fcs_bgzf_index walks the members of comp[0, comp_bytes) (gzip header with
 * the BC extra field, payload, CRC32, ISIZE), stopping before an incomplete
 * member or after cap members: coff[0..n] = member starts (coff[n] = bytes of
 * whole members = *comp_used), uoff[0..n] = their inflated starts (prefix sums
 * of ISIZE).  FCS_ERR_INVALID when the bytes at a member start are not a
 * BGZF header.
 *
 * fcs_bgzf_inflate: host buffers; inflates the whole members of comp into
 * out (concatenated), *out_bytes = their inflated size (FCS_ERR_INVALID when it
 * exceeds out_cap, or when a member is corrupt / fails its CRC: the message
 * names the member).  A trailing incomplete member is left for the next call
 * (*comp_used tells where it starts).
 *
 * fcs_bgzf_inflate_dev: device buffers, stream-ordered; dev_coff / dev_uoff
 * as fcs_bgzf_index returns them, dev_status[k] = FCS_BGZF_* of member k
 * (member k's output range holds its bytes when it is FCS_BGZF_OK; a failing
 * member may leave partial bytes there, never outside its range). */
#define FCS_BGZF_OK 0
#define FCS_BGZF_CORRUPT 1  /* bad DEFLATE stream, header or ISIZE */
#define FCS_BGZF_OVERFLOW 2 /* the stream inflates past ISIZE */
#define FCS_BGZF_CRC 3      /* CRC-32 mismatch */
int fcs_bgzf_index(const uint8_t* comp, int64_t comp_bytes, int64_t* coff, int64_t* uoff, int32_t cap,
                   int32_t* n_members, int64_t* comp_used);
int fcs_bgzf_inflate(const uint8_t* comp, int64_t comp_bytes, uint8_t* out, int64_t out_cap, int64_t* comp_used,
                     int64_t* out_bytes, int32_t device);
int fcs_bgzf_inflate_dev(const uint8_t* dev_comp, const int64_t* dev_coff, const int64_t* dev_uoff, int32_t n,
                         uint8_t* dev_out, int32_t* dev_status, int32_t device, void* stream);
/* fcs_bgzf_inflate without waiting: FCS_BGZF_BUSY (nothing done, *comp_used =
 * 0) unless an inflate session is idle whose staging arenas already hold the
 * call, so a reader can inflate on its own cores instead of queueing.
 * fcs_bgzf_warmup creates `sessions` inflate sessions with `arena_bytes` of
 * pinned host and device staging each (the growth a first call would pay). */
#define FCS_BGZF_BUSY 1
int fcs_bgzf_inflate_try(const uint8_t* comp, int64_t comp_bytes, uint8_t* out, int64_t out_cap, int64_t* comp_used,
                         int64_t* out_bytes, int32_t device);
int fcs_bgzf_warmup(int32_t device, int32_t sessions, int64_t arena_bytes);

/* ---------------------------------------------- synthetic workload builders */
/* Seeded generators for the benchmark configurations (BASELINE.json C2/C3).
 * Deterministic for a given seed.  Callers size the buffers with the *_sizes
 * functions first. */

/* C2: n_pairs independent pairs, read length R, hap length uniform in
 * [hmin, hmax]; read = hap substring with 1% substitutions and 0.1% 1-3 bp
 * indels; base_q uniform [10,40], ins_q = del_q = 45, gcp = 10.  One read and
 * one hap per pair (pair p = (p, p)).  Reads may come out shorter than R when
 * the source window runs off the hap; lengths are written to read_len. */
int fcs_synth_phmm_sizes(uint64_t seed, int64_t n_pairs, int32_t R, int32_t hmin, int32_t hmax,
                         int64_t* read_bytes, int64_t* hap_bytes);
int fcs_synth_phmm(uint64_t seed, int64_t n_pairs, int32_t R, int32_t hmin, int32_t hmax,
                   uint8_t* read_bases, uint8_t* read_bq, uint8_t* read_iq, uint8_t* read_dq,
                   uint8_t* read_gcp, int64_t* read_off, int32_t* read_len, uint8_t* hap_bases,
                   int64_t* hap_off, int32_t* hap_len);

/* C3: reads of length read_len sampled from a random reference of ref_len
 * bases (0.5% substitutions, 0.05% indels), one seed per read; emits the left
 * (reversed) and right extension tasks a bwa-mem seed produces, with
 * tlen = min(qlen + w, available reference).  mode 1 instead emits fixed
 * qlen=fixed_q / tlen=fixed_t tasks (clean GCUPS variant).  Returns the task
 * count in *n_tasks (≤ 2 * n_reads). */
int fcs_synth_bsw_sizes(uint64_t seed, int64_t n_reads, int32_t read_len, int64_t ref_len, int32_t w,
                        int32_t mode, int32_t fixed_q, int32_t fixed_t, int64_t* n_tasks,
                        int64_t* qbytes, int64_t* tbytes);
int fcs_synth_bsw(uint64_t seed, int64_t n_reads, int32_t read_len, int64_t ref_len, int32_t w,
                  int32_t mode, int32_t fixed_q, int32_t fixed_t, uint8_t* qbuf, int64_t* qoff,
                  int32_t* qlen, uint8_t* tbuf, int64_t* toff, int32_t* tlen, int32_t* h0,
                  int32_t* wv, int64_t* n_tasks);

#ifdef __cplusplus
}
#endif

#endif /* FCSHIP_H */
