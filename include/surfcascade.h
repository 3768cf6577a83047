/*
 * surfcascade.h -- C ABI of the MI355X-native SURF-cascade detect path.
 *
 * The reference (mrgloom/SurfCascade) has no FFI; its de-facto API is the
 * in-process C++ classes used by ObjDetector's --detect branch.  Each entry
 * point below names the reference interface it replaces:
 *
 *   Model(string cfg) + Model::Load(CascadeClassifier&)   Model.h:15-18,
 *                                                          Model.cpp:97-194
 *   Model::Save(CascadeClassifier&)                        Model.cpp:21-95
 *   StageClassifier::theta, LogisticRegression::{w,        StageClassifier.h:24,
 *     patch_index, model_->bias}                           LogisticRegression.h:16-21
 *   CascadeClassifier::GetFittedPatchIndexes               CascadeClassifier.cpp:83-91
 *   DenseSURFFeatureExtractor::ExtractPatches              DenseSURFFeatureExtractor.cpp:49-63
 *   DenseSURFFeatureExtractor::IntegralImage + the scan    DenseSURFFeatureExtractor.cpp:65-87,
 *     loop (sum / ProjectPatches / CalcFeature /           ObjDetector.cpp:160-220
 *     CascadeClassifier::Predict2) for one image
 *
 * Conventions: every function returns an int status (SC_OK = 0, negative =
 * error class) and sets a thread-local message readable via sc_last_error();
 * no C++ exception crosses the ABI.  The caller owns input and output
 * buffers; the library owns device memory.  One HIP stream per detector;
 * distinct detectors may be used from different threads, one detector is not
 * thread-safe.  Raw windows come back sorted by (frame, level, y, x) -- the
 * reference's own order is nondeterministic (omp critical, ObjDetector.cpp:205).
 * Model loading is strict: a missing key or a type mismatch is an error
 * (the reference silently keeps a partial cascade, Model.cpp:188-191).
 */
#ifndef SURFCASCADE_H
#define SURFCASCADE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SC_OK 0
#define SC_ERR_INVALID (-1)  /* bad argument / unsupported geometry         */
#define SC_ERR_IO (-2)       /* file I/O        (Model.cpp:106-110)         */
#define SC_ERR_PARSE (-3)    /* syntax          (Model.cpp:111-116)         */
#define SC_ERR_MODEL (-4)    /* missing key or type mismatch                */
#define SC_ERR_DEVICE (-5)   /* HIP runtime error / no usable gfx950 device */
#define SC_ERR_CAPACITY (-6) /* output too small; *n_out = required count   */
#define SC_ERR_NOMEM (-7)

typedef struct sc_model sc_model;
typedef struct sc_detector sc_detector;

/* Scan parameters; defaults are the reference's compile-time constants. */
typedef struct {
    int base_len;        /* 70    window side at level 0 (ObjDetector.cpp:104) */
    double scale_factor; /* 1.1   l_i = (int)(base_len*pow(1.1,i)) (:180)      */
    int n_levels;        /* -1 => (int)min(log(W/70f)/log1.1, ...)+1 (:174)    */
    int step;            /* 0  => base_len>20 ? base_len/20 : 1 (:139)         */
    float prefilter_k;   /* 6     sum(win) > area*6 (:188)                     */
    double stride_score; /* 0.5   multi = score<0.5 ? 2 : 1 (:214)             */
    int tmpl_w, tmpl_h;  /* 40x40 template (:112)                              */
    int aspect_h;        /* 1; window height = aspect_h*l (2 for 64x128 ext.)  */
} sc_scan_params;

/* One raw (pre-groupRectangles) detection, ObjDetector.cpp:203-208. */
typedef struct {
    int32_t level, x, y, w, h;
    int32_t stage_reached; /* == number of stages for a detection          */
    double score;          /* ((double)s_last + p + 1) / S  (:201)          */
} sc_window;

/* Device-side record written by sc_enqueue_device (40 bytes). */
typedef struct {
    int32_t frame, level, x, y, w, h, stage_reached, _pad;
    double score;
} sc_det_record;

void sc_scan_params_default(sc_scan_params *p);

/* ---- model (Model.cpp) ------------------------------------------------- */
int sc_model_load(const char *cfg_path, sc_model **out);
int sc_model_parse(const char *text, size_t len, sc_model **out);
int sc_model_save(const sc_model *m, const char *cfg_path);
int sc_model_num_stages(const sc_model *m);
int sc_model_stage(const sc_model *m, int stage, float *theta, int *n_weak);
int sc_model_weak(const sc_model *m, int stage, int k, int *patch_index,
                  float w33[33], double *bias);
void sc_model_free(sc_model *m);

/* ---- template patches (DenseSURFFeatureExtractor::ExtractPatches) ------- */
int sc_extract_patches(int tmpl_w, int tmpl_h, int32_t *rects_xywh, int cap);

/* ---- detector ----------------------------------------------------------- */
int sc_detector_create(const char *cfg_path, const sc_scan_params *p,
                       int device, sc_detector **out);
int sc_detector_create_from_model(const sc_model *m, const sc_scan_params *p,
                                  int device, sc_detector **out);
void sc_detector_destroy(sc_detector *d);

/* One host frame -> raw windows (sorted).  *n_out = total count even when it
 * exceeds capacity (then SC_ERR_CAPACITY and the first `capacity` stored).
 * Frames are 2x2 .. 32767x32767; one smaller than the base window scans no
 * level and returns no window (the reference's level loop runs zero times,
 * ObjDetector.cpp:174-178). */
int sc_detect(sc_detector *d, const uint8_t *gray, int w, int h,
              int stride_bytes, sc_window *out, int capacity, int *n_out);
/* n host frames of one size.  out holds all frames' windows back to back;
 * n_out[f] = count for frame f. */
int sc_detect_batch(sc_detector *d, const uint8_t *const *frames, int n,
                    int w, int h, int stride_bytes, sc_window *out,
                    int capacity, int *n_out);
/* n frames already in device memory (frame f at d_frames + f*h*stride). */
int sc_detect_device(sc_detector *d, const uint8_t *d_frames, int n, int w,
                     int h, int stride_bytes, sc_window *out, int capacity,
                     int *n_out);
/* Window-grid sharding of every frame over `world` ranks (SURVEY.md 8e:
 * single-frame 1/2/4/8-GPU runs).  This detector then evaluates only the
 * (level, y) rows i of the canonical row list (level-major, y ascending)
 * with i % world == rank; the adaptive-stride x chain never leaves its row
 * (ObjDetector.cpp:185-217), so the union over ranks of the raw windows is
 * exactly the unsharded result.  The reference has no multi-device path; the
 * closest thing is its OpenMP split over levels (ObjDetector.cpp:177).
 * (rank 0, world 1) restores the whole grid. */
int sc_detector_set_shard(sc_detector *d, int rank, int world);
/* Asynchronous form on the detector's stream: device records (unsorted;
 * canonical order = sort by frame, level, y, x) + device counters
 * d_counts[0] = total, d_counts[1+f] = frame f's count.  No host sync. */
int sc_enqueue_device(sc_detector *d, const uint8_t *d_frames, int n, int w,
                      int h, int stride_bytes, sc_det_record *d_out,
                      int capacity, int32_t *d_counts);
int sc_synchronize(sc_detector *d);
void *sc_detector_stream(sc_detector *d); /* hipStream_t */
/* Stream ordering of the device-memory entry points (sc_detect_device,
 * sc_enqueue_device, sc_mine_device).  They run on the detector's own
 * non-blocking stream, which is NOT ordered against the caller's streams:
 *  - before handing over device frames / output buffers that work on another
 *    stream still writes (or frees and re-uses), call
 *    sc_detector_wait_stream(d, that_stream): the detector's next work waits
 *    for everything already queued there (no host sync);
 *  - before reading sc_enqueue_device's outputs on another stream, call
 *    sc_stream_wait_detector(d, that_stream), or sc_synchronize(d).
 * Device pointers must be device memory of the detector's GPU (checked:
 * SC_ERR_INVALID otherwise). */
int sc_detector_wait_stream(sc_detector *d, void *stream);
int sc_stream_wait_detector(sc_detector *d, void *stream);
/* Launch on the caller's stream instead (a stream of the detector's GPU, NULL
 * = HIP's null stream), or back on the detector's own (use_own != 0, stream
 * ignored).  Work on the caller's stream is then ordered with the detector's
 * without the two calls above (one event pair less per call).  The switch is
 * ordered: work queued after it waits for the detector's work queued before
 * it.  The caller keeps the stream alive while it is set. */
int sc_detector_set_stream(sc_detector *d, void *stream, int use_own);

/* ---- hard-negative mining (training side) ----------
 * DenseSURFFeatureExtractor::FillNegSamples' scan of one negative image
 * (DenseSURFFeatureExtractor.cpp:124-195): square windows l_k =
 * (int)(tmpl_w * 1.1^k) for k = 0..(int)min(log(W/(float)tmpl_w)/log 1.1,
 * log(H/(float)tmpl_w)/log 1.1), rows and columns at stride 10, no
 * prefilter.  A window is a candidate (a false positive to train on) when
 * the cascade accepts it (CascadeClassifier::Predict, CascadeClassifier.cpp:
 * 63-72); m == NULL is the first round (no stage yet): every window is.
 * The miner is an sc_detector; sc_detect* on it fail with SC_ERR_INVALID. */
int sc_miner_create(const sc_model *m, int tmpl_w, int tmpl_h, int device,
                    sc_detector **out);
/* Candidates in (level, y, x) order -- the reference appends them from
 * OpenMP threads in a nondeterministic order and stops at n_total.  The first
 * `capacity` go to wins (stage_reached = number of stages, score = last
 * stage score) and, when features != NULL, their ExtractFeatures descriptors
 * over every template patch (sc_extract_patches order, CalcFeature +
 * Normalize, :88-93, :379-457): float[capacity][n_patches][32].
 * *n_out = all candidates; SC_ERR_CAPACITY when that exceeds capacity. */
int sc_mine(sc_detector *d, const uint8_t *gray, int w, int h, int stride_bytes,
            sc_window *wins, float *features, int capacity, int *n_out);
/* sc_mine on a frame already in device memory, the descriptors written
 * straight into d_features (device memory, float[capacity][n_patches][32], or
 * NULL): no host copy of the descriptors, which dominates sc_mine when many
 * are kept (FillNegSamples' sample matrix, DenseSURFFeatureExtractor.cpp:
 * 124-195, stays on the GPU for the trainer).  Windows still go to the host. */
int sc_mine_device(sc_detector *d, const uint8_t *d_gray, int w, int h, int stride_bytes,
                   sc_window *wins, float *d_features, int capacity, int *n_out);
/* FillNegSamples over n negative images of one size in one pass (the
 * reference loops over its image list, DenseSURFFeatureExtractor.cpp:
 * 132-190): candidates in (image, level, y, x) order, the first `capacity`
 * of the whole batch kept, windows back to back; n_out[f] = image f's
 * candidates (all of them, kept or not).  sc_mine is the n = 1 case.  The
 * device form takes n frames at d_frames + f*h*stride and writes the
 * descriptors to device memory, as sc_mine_device. */
int sc_mine_batch(sc_detector *d, const uint8_t *const *frames, int n, int w, int h,
                  int stride_bytes, sc_window *wins, float *features, int capacity,
                  int *n_out);
int sc_mine_batch_device(sc_detector *d, const uint8_t *d_frames, int n, int w, int h,
                         int stride_bytes, sc_window *wins, float *d_features, int capacity,
                         int *n_out);

/* ---- introspection / parity dumps -------------------------------------- */
#define SC_INFO_LEVELS 1        /* levels used for the last geometry         */
#define SC_INFO_GRID_WINDOWS 2  /* stride-step grid windows per frame        */
#define SC_INFO_ROWS 3          /* (level, y) rows per frame                 */
#define SC_INFO_TABLE_PITCH 4   /* integral-table row pitch in cells         */
#define SC_INFO_VISITED 5       /* windows the adaptive stride visited (last) */
#define SC_INFO_FUSED_FRAMES 6  /* frames of the last call whose integral      */
                                /* column walks ran inside the chain kernel    */
#define SC_INFO_CHAIN_WAVES 7   /* waves per workgroup of the last chain-kernel */
                                /* launch (8, 10, 12, 14 or 16; 0: none yet)   */
#define SC_INFO_COLUMN_PASS 8   /* the last call's integral column pass for the */
                                /* frames built outside the chain kernel:      */
                                /* 1 two-pass (rowcarry R + colsum), 2 colstrip,*/
                                /* 3 two-pass in row segments (one frame)      */
#define SC_INFO_SPEC_ROUNDS 9   /* speculative evaluation rounds of the last    */
                                /* chain launch (one-frame launches only)      */
#define SC_INFO_CHAIN_SUBQ 10   /* dequeue sub-queues per XCD of the last chain  */
                                /* launch (4 one-frame launches, 1 batches)    */
#define SC_INFO_ITEM_FORM 11    /* integral cells and item form of the current */
                                /* geometry: 1 channel-split cells, one lane   */
                                /* per item; 2 interleaved 32-B cells, the     */
                                /* lane-pair item form (sc_device.hpp)         */
int sc_detector_info(sc_detector *d, int what, int64_t *value);

/* ---- tuning and test options ---------------------------------------------
 * Options 1-14, 17-19 and 21 are schedule / layout choices that never change a result bit
 * (tests/test_gpu_parity.py runs each against the oracle); the defaults are
 * the measured-fastest.  Options 15-16 restrict the scan to a range of levels
 * (profiling of level groups): they DO change the result, to the windows of
 * those levels.  Options 20 and 22 are test hooks (a deliberately lost
 * hand-off or walk count: the call must fail, tests/test_gpu_configs.py).  The library reads no
 * environment variable: these are set per detector, explicitly. */
#define SC_OPT_FULL_GRID 1    /* 1: evaluate every grid window (cascade + walk   */
                              /* kernels) instead of the lazy chain kernel (0) */
#define SC_OPT_CHUNK_MIN 2    /* stages with >= this many survivors run one lane */
                              /* per window (0: only stages whose weak count   */
                              /* exceeds the item buffer)                      */
#define SC_OPT_TABLE_LAYOUT 3 /* integral cells: 0 channel-split halves,       */
                              /* 1 interleaved 32-B cells                      */
#define SC_OPT_PHASES 4       /* phase planes per step: 0 auto (lazy 2, full 1) */
#define SC_OPT_SUBSTRIPS 5    /* full grid: strips per XCD band (0 auto)       */
#define SC_OPT_BAND_ROWS 6    /* full grid: grid rows per task band (0: 1)     */
#define SC_OPT_ROW_ORDER 7    /* chain tasks: 0 level-major, 1 y-major,        */
                              /* 2 blocks of ROW_BLOCK grid rows (default),    */
                              /* 3 the same blocks bottom-up                   */
#define SC_OPT_ROW_BLOCK 8    /* grid rows per block (default 32)              */
#define SC_OPT_CHAIN_CHUNK 9  /* frames per chain-kernel launch at most (0:    */
                              /* as many as 32-bit table offsets allow)        */
#define SC_OPT_LDS_WEIGHTS 10 /* -1 auto, 0 weights through the caches, 1 LDS  */
#define SC_OPT_WGS_PER_CU 11  /* workgroups per CU, 0 = occupancy limit        */
#define SC_OPT_PROFILE 12     /* chain-kernel phase counters (profiling builds) */
#define SC_OPT_CHAIN_SEGS 13  /* chain kernel: segments per row (0 auto: 4 for a */
                              /* one-frame launch of fewer than 8 grid shards, */
                              /* else 8; or 1, 2, 4, 8)                        */
#define SC_OPT_INTEGRAL_PASSES 14 /* integral: 0 auto (two passes up to 3     */
                              /* frames), 1 colstrip, 2 rowfull + colsum       */
#define SC_OPT_LEVEL_LO 15    /* scan only levels >= LEVEL_LO (default 0)      */
#define SC_OPT_LEVEL_HI 16    /* ... and < LEVEL_HI (0: every level)           */
#define SC_OPT_CHAIN_WAVES 17 /* chain kernel waves per CU: 0 auto (16 when the  */
                              /* model and their scratch fit the LDS, a        */
                              /* frame's table is <= 128 MiB and the launch    */
                              /* has 2+ frames; 10 for tables > 128 MiB with   */
                              /* 2+ frames; else 12), or 8, 10, 12, 14, 16     */
#define SC_OPT_INTEGRAL_FUSE 18 /* integral column walks inside the chain      */
                              /* kernel: 0 auto (from 4 frames per launch),   */
                              /* 1 never, 2 whenever a launch has 2+ frames    */
#define SC_OPT_INTEGRAL_PRE 19 /* fused: frames per launch integrated before   */
                              /* the chain kernel (0: default 2; 1 for tables  */
                              /* > 128 MiB)                                    */
#define SC_OPT_TEST_DROP_HANDOFF 20 /* test only (-1 off): the chain kernel drops */
                              /* the segment-0 hand-off of row task `value`  */
                              /* of every launch; the watchdog must then     */
                              /* raise SC_ERR_DEVICE at the next sync.  Only */
                              /* the test-hook build (lib/testhooks) accepts */
                              /* a value other than -1                       */
#define SC_OPT_CHAIN_SUBQ 21  /* chain kernel dequeue counters per XCD queue: */
                              /* 0 auto (4 for a one-frame launch, else 1),    */
                              /* or 1..8                                       */
#define SC_OPT_TEST_DROP_WALK 22 /* test only (-1 off): the fused column walk  */
                              /* `value` of every launch does not count itself */
                              /* done; tasks waiting for that frame's table    */
                              /* must time out and the next sync raise         */
                              /* SC_ERR_DEVICE (test-hook build only)          */
#define SC_OPT_CHAIN_SPEC 23  /* one-frame chain launches: speculative rounds */
                              /* (2 x 128 windows each) per waiting segment    */
                              /* task: 0 auto (1 for a whole frame, the whole  */
                              /* segment for a grid shard), or 1..64           */
#define SC_OPT_CHAIN_SLOTS 24 /* chain kernel task slots per wave: 0 auto (1   */
                              /* for a one-frame launch, 2 for batches), 1, 2  */
int sc_detector_set_option(sc_detector *d, int option, int64_t value);

/* Enable per-window debug records (grid order) for the next detect calls. */
int sc_detector_set_debug(sc_detector *d, int on);
#define SC_DUMP_INTEGRAL 1    /* float[(H+1)*(W+1)*8] of frame `frame`       */
#define SC_DUMP_GRID_STAGE 2  /* int16[grid]: p (-1 = prefilter reject, -2 =  */
                              /* not evaluated: the default lazy grid only   */
                              /* evaluates windows the x chain reaches)      */
#define SC_DUMP_GRID_SCORE 3  /* float[grid]: last stage score               */
#define SC_DUMP_GRID_VISIT 4  /* uint8[grid]: 1 = visited by the x chain     */
int sc_debug_dump(sc_detector *d, int what, int frame, void *dst,
                  size_t bytes);

/* Per-kernel HIP-event timing on the detector's stream (bench / profiling). */
#define SC_KERNEL_ROWSCAN 0
#define SC_KERNEL_COLSCAN 1
#define SC_KERNEL_WINDOWS 2 /* prefilter + cascade */
#define SC_KERNEL_WALK 3    /* adaptive-stride walk + detections */
#define SC_KERNEL_COUNT 4
int sc_set_timing(sc_detector *d, int on);
int sc_get_timing(sc_detector *d, double ms_total[SC_KERNEL_COUNT],
                  int64_t launches[SC_KERNEL_COUNT]);

/* ---- post-processing (ObjDetector.cpp:223-231) --------------------------
 * cv::groupRectangles(wins, weights = 0s, levelWeights = scores, 2, 0.2)
 * (OpenCV 3.0.0 objdetect, called at ObjDetector.cpp:224-225) and the FDDB
 * text block the reference writes per image (:228-231). */
typedef struct {
    int32_t x, y, width, height; /* cv::Rect                                 */
    double score;                /* levelWeight: the cluster's best score    */
} sc_scored_rect;

/* Cluster rectangles (SimilarRects(eps) components), keep clusters with more
 * than group_threshold members that are not inside a better-supported one;
 * each output is the members' mean rectangle with their maximum score.
 * *n_out = output count (SC_ERR_CAPACITY when it exceeds capacity). */
int sc_group_rectangles(const sc_scored_rect *in, int n, int group_threshold,
                        double eps, sc_scored_rect *out, int capacity,
                        int *n_out);
/* The same per frame over raw detection records of n_frames frames (any
 * order; each frame's rectangles enter in canonical (level, y, x) order).
 * Frames' results back to back in out; frame_counts[f] = frame f's count. */
int sc_group_detections(const sc_det_record *rec, int n, int n_frames,
                        int group_threshold, double eps, sc_scored_rect *out,
                        int capacity, int32_t *frame_counts, int *n_out);
/* "name\ncount\nx y w h score\n..." (std::ostream default double format).
 * *len = bytes needed (excluding NUL); SC_ERR_CAPACITY if cap <= *len. */
int sc_fddb_format(const char *image_name, const sc_scored_rect *r, int n,
                   char *buf, size_t cap, size_t *len);

/* fast_nms (ObjDetector.cpp:318-383), the reference's commented-out
 * alternative to groupRectangles (:223): greedy suppression of every
 * rectangle whose (w+1)(h+1)-normalised overlap with the current best
 * exceeds overlap_th, in the reference's exact tie order (its exchange sort,
 * :275-288, is reproduced as written: O(n^2)).  out = picked rectangles in
 * pick order (best score first); SC_ERR_CAPACITY when *n_out > capacity. */
int sc_fast_nms(const sc_scored_rect *in, int n, double overlap_th,
                sc_scored_rect *out, int capacity, int *n_out);

/* ---- input side (ObjDetector.cpp:164) -----------------------------------
 * cv::imread(path, cv::IMREAD_GRAYSCALE) for JPEG files: baseline,
 * extended-sequential and progressive Huffman JPEG, 8-bit, 1 or 3 components
 * (luma, as libjpeg's JCS_GRAYSCALE output: JDCT_ISLOW inverse DCT).  Writes
 * a w x h plane with row stride w.  *w / *h are set even when the buffer is
 * too small (SC_ERR_CAPACITY), so a NULL / 0 call sizes the buffer.
 * SC_ERR_PARSE: not a JPEG, an unsupported coding process, a corrupt
 * Huffman table, or more than 2^28 pixels (twice what a detector accepts). */
int sc_decode_jpeg_gray(const uint8_t *data, size_t len, uint8_t *out,
                        size_t cap, int *w, int *h);
int sc_imread_gray(const char *path, uint8_t *out, size_t cap, int *w,
                   int *h);

/* ---- device self-check of the Normalize arithmetic ----------------------
 * The item loop's Normalize (DenseSURFFeatureExtractor.cpp:427-457) uses a
 * shortened IEEE sqrt and reciprocal (sc_device.hpp sqrt_rn / rcp_rn).  This
 * runs every f32 bit pattern in [lo_bits, hi_bits] through the short
 * sequence (op 0: sqrt, 1: reciprocal), the compiler's full IEEE sequence and
 * the f64 route on GPU `device`; out[0] = patterns differing from the full
 * sequence, out[1] = from the f64 route, out[2] = patterns checked, out[3] =
 * the smallest differing pattern (UINT64_MAX: none).  Test support: the
 * detect path does not call it. */
int sc_selftest_rn(int device, int op, uint32_t lo_bits, uint32_t hi_bits,
                   uint64_t out[4]);
/* Operand ranges Normalize can produce for the largest accepted frame
 * (|box sum| <= 2*255*W*H): ss[0..1] bounds SS and SS2, d[0..1] bounds
 * sqrt(SS2); the frame limits of sc_detect* keep these inside the ranges
 * sc_selftest_rn is run over (tests/test_gpu_rn.py). */
void sc_normalize_operand_range(int max_w, int max_h, double ss[2], double d[2]);

const char *sc_last_error(void);
const char *sc_version(void);
/* What this library was built from, as one JSON object: "build_id" (sha256
 * prefix over every csrc/ source, this header, the Makefile and the extra
 * -D flags), "flags" (those -D flags), "arch", and whether it is a timing
 * "ablation" build (wrong results possible), a "test_hooks" build or a
 * "profiling" build.  The product library reports flags "" and all three
 * false (tests/test_abi.py).  No reference counterpart: measurement
 * provenance (bench.py stamps its line and the PMC table with build_id). */
const char *sc_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* SURFCASCADE_H */
