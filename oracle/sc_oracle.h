/*
 * sc_oracle.h -- CPU restatement of the SurfCascade detect path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (libsurfcascade.so) never
 * links, loads or calls it.
 *
 * Parity status: the reference cannot be built here (needs OpenCV 3.0.0,
 * Win32, MSVC-only intrinsics) and executing it was DENIED by the environment
 * (SURVEY.md 8c).  This restatement is written from the reference source text
 * and pinned by hand-derivable known-answer tests (tests/test_oracle_kat.py);
 * third-party arithmetic (OpenCV cv::integral 8U->32F, MSVC CRT exp) follows
 * the published scalar algorithms: "parity unpinned" for those two pieces.
 *
 * Every function cites the reference file:line it restates; paths are
 * relative to the reference root (ObjDetector/...).
 */
#ifndef SC_ORACLE_H
#define SC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Flattened cascade: stages in order, weak classifiers in stage order. */
typedef struct {
    int n_stages;
    const int32_t *n_weak;  /* [n_stages]                                   */
    const float *theta;     /* [n_stages]       StageClassifier.h:24         */
    const int32_t *patch;   /* [total_weak*4]   template rect x,y,w,h of the */
                            /*                  weak's patch_index           */
    const float *w;         /* [total_weak*33]  LogisticRegression.h:18      */
    const double *bias;     /* [total_weak]     liblinear model::bias        */
    int tmpl_w, tmpl_h;     /* 40x40 (ObjDetector.cpp:112)                   */
} sco_model;

typedef struct {
    int base_len;        /* 70   ObjDetector.cpp:104                          */
    int aspect_h;        /* 1    window height = aspect_h * l (build ext.)    */
    int n_levels;        /* <0 : reference formula ObjDetector.cpp:174        */
    int step;            /* <=0: base_len>20 ? base_len/20 : 1  (:139)        */
    float prefilter_k;   /* 6    ObjDetector.cpp:188                          */
    double stride_score; /* 0.5  ObjDetector.cpp:214                          */
} sco_params;

/* One raw (pre-grouping) detection window; 32 bytes. */
typedef struct {
    int32_t level, x, y, w, h, stage;
    double score;
} sco_window;

int sco_level_len(int base, int i);
int sco_num_levels(int W, int H, int base_w, int base_h);
int sco_step(const sco_params *p);
int sco_effective_levels(int W, int H, const sco_params *p);
int64_t sco_grid_count(int W, int H, const sco_params *p);

int sco_extract_patches(int tw, int th, int32_t *rects, int cap);

void sco_gradients(const uint8_t *img, int W, int H, int stride, uint8_t *grad);
void sco_integral(const uint8_t *img, int W, int H, int stride, float *T);

int sco_prefilter(const float *T, int W, int x, int y, int w, int h, float k,
                  float *m_out);
void sco_project(const int32_t tr[4], float scale, int wx, int wy,
                 int32_t out[4]);
void sco_normalize(float f[32]);
void sco_calc_feature(const float *T, int W, const int32_t rect[4],
                      float f[32]);
float sco_lr_predict(const float *w33, double bias, const float f[32]);

int sco_eval_window(const float *T, int W, const sco_model *m, int l, int lh,
                    int x, int y, float k, float *s_last,
                    float *stage_scores);
void sco_all_stage_scores(const float *T, int W, const sco_model *m, int l,
                          int x, int y, float *stage_scores);

void sco_stage_score_batch(const float *T, int W, const sco_model *m,
                           const int32_t *l, const int32_t *x, const int32_t *y,
                           int64_t n, int stage, float *out, int nthreads);
int64_t sco_eval_grid(const float *T, int W, int H, const sco_model *m,
                      const sco_params *p, int16_t *p_out, float *s_out,
                      int nthreads);
int64_t sco_detect(const float *T, int W, int H, const sco_model *m,
                   const sco_params *p, sco_window *out, int64_t cap,
                   int64_t *n_visited, int nthreads);
int64_t sco_walk_grid(const int16_t *p_grid, const float *s_grid, const int64_t *layout,
                      int n_levels, int n_stages, double stride_score, uint8_t *visited);
void sco_exposure(const float *T, int W, int H, const sco_model *m, const sco_params *p,
                  int64_t st[8], int nthreads);
/* exp() sensitivity of the visited windows (VERDICT r2 Next 6): counters in
 * sc_oracle.c; zd receives the z of the first zcap flipping evaluations. */
void sco_exp_sensitivity(const float *T, int W, int H, const sco_model *m, const sco_params *p,
                         int64_t st[9], double *zd, int64_t zcap, int nthreads);
int64_t sco_detect_frame(const uint8_t *img, int W, int H, int stride,
                         const sco_model *m, const sco_params *p,
                         sco_window *out, int64_t cap, int64_t *n_visited,
                         int nthreads, float *scratch_T);

/* Hard-negative scan of one image (FillNegSamples): candidates + descriptors. */
int64_t sco_mine(const float *T, int W, int H, const sco_model *m, const int32_t *patches,
                 int n_patches, sco_window *out, float *feat, int64_t cap, int nthreads);

/* Post-processing (sc_oracle_group.c): groupRectangles + FDDB block. */
typedef struct {
    int32_t x, y, w, h;
    double score;
} sco_rect;

int sco_group_rectangles(const sco_rect *in, int n, int group_threshold, double eps,
                         sco_rect *out);
long sco_fddb_format(const char *name, const sco_rect *r, int n, char *buf, long cap);

#ifdef __cplusplus
}
#endif
#endif
