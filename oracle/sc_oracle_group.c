/*
 * sc_oracle_group.c -- CPU restatement of the reference's post-processing:
 * cv::groupRectangles(wins, weights = 0s, levelWeights = scores, 2, 0.2) and
 * the FDDB text writer (ObjDetector.cpp:223-231).
 *
 * TEST INFRASTRUCTURE ONLY (see sc_oracle.h).
 *
 * groupRectangles lives in OpenCV 3.0.0 objdetect (cascadedetect.cpp), an
 * un-vendored dependency of the reference (OpenCV_Release.props:11).  This
 * restates its published algorithm: cv::partition (union-find with rank and
 * path compression, classes numbered by first appearance) under the
 * SimilarRects(eps) predicate, per-class mean rectangles, the per-class
 * maximum levelWeight among members with the maximal rejectLevel, the
 * "> groupThreshold members" filter and the "small rectangle inside a large
 * one" filter.  No OpenCV output is available here to pin it: parity
 * unpinned (tests/test_group.py holds hand-derived known answers).
 */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sc_oracle.h"

/* SimilarRects::operator() (cascadedetect.hpp) */
static int similar(const sco_rect *a, const sco_rect *b, double eps) {
    int mw = a->w < b->w ? a->w : b->w, mh = a->h < b->h ? a->h : b->h;
    double delta = eps * (mw + mh) * 0.5;
    return abs(a->x - b->x) <= delta && abs(a->y - b->y) <= delta &&
           abs(a->x + a->w - b->x - b->w) <= delta && abs(a->y + a->h - b->y - b->h) <= delta;
}

/* cv::partition (core/operations.hpp): returns the class count; labels[i]. */
static int partition(const sco_rect *r, int n, double eps, int *labels) {
    int *parent = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    int *rank = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        parent[i] = -1;
        rank[i] = 0;
    }
    for (int i = 0; i < n; i++) {
        int root = i;
        while (parent[root] >= 0) root = parent[root];
        for (int j = 0; j < n; j++) {
            if (i == j || !similar(&r[i], &r[j], eps)) continue;
            int root2 = j;
            while (parent[root2] >= 0) root2 = parent[root2];
            if (root2 != root) {
                int rk = rank[root], rk2 = rank[root2];
                if (rk > rk2) {
                    parent[root2] = root;
                } else {
                    parent[root] = root2;
                    rank[root2] += rk == rk2;
                    root = root2;
                }
                int k = j, p;
                while ((p = parent[k]) >= 0) {
                    parent[k] = root;
                    k = p;
                }
                k = i;
                while ((p = parent[k]) >= 0) {
                    parent[k] = root;
                    k = p;
                }
            }
        }
    }
    int nclasses = 0;
    for (int i = 0; i < n; i++) {
        int root = i;
        while (parent[root] >= 0) root = parent[root];
        if (rank[root] >= 0) rank[root] = ~nclasses++;
        labels[i] = ~rank[root];
    }
    free(parent);
    free(rank);
    return nclasses;
}

/* cvRound / saturate_cast<int>: round to nearest, ties to even (SSE2 cvt) */
static int round_f(float v) { return (int)lrintf(v); }
static int round_d(double v) { return (int)lrint(v); }

/* groupRectangles(rectList, groupThreshold, eps, &weights, &levelWeights)
 * with weights all 0 and levelWeights = scores (ObjDetector.cpp:224-225).
 * in/out may not alias; returns the number of output rectangles. */
int sco_group_rectangles(const sco_rect *in, int n, int group_threshold, double eps,
                         sco_rect *out) {
    if (group_threshold <= 0 || n == 0) {
        if (n > 0) memcpy(out, in, sizeof(sco_rect) * (size_t)n);
        return n;
    }
    int *labels = (int *)malloc(sizeof(int) * (size_t)n);
    int nc = partition(in, n, eps, labels);
    long long *sx = (long long *)calloc((size_t)nc * 4, sizeof(long long));
    int *cnt = (int *)calloc((size_t)nc, sizeof(int));
    int *rlev = (int *)calloc((size_t)nc, sizeof(int));
    double *rw = (double *)malloc(sizeof(double) * (size_t)nc);
    sco_rect *rr = (sco_rect *)malloc(sizeof(sco_rect) * (size_t)nc);
    for (int c = 0; c < nc; c++) rw[c] = DBL_MIN;
    for (int i = 0; i < n; i++) {
        int c = labels[i];
        sx[4 * c + 0] += in[i].x;
        sx[4 * c + 1] += in[i].y;
        sx[4 * c + 2] += in[i].w;
        sx[4 * c + 3] += in[i].h;
        cnt[c]++;
    }
    for (int i = 0; i < n; i++) {  /* weights[i] == 0 == rejectLevels[c]: max levelWeight */
        int c = labels[i];
        if (0 > rlev[c]) {
            rlev[c] = 0;
            rw[c] = in[i].score;
        } else if (0 == rlev[c] && in[i].score > rw[c]) {
            rw[c] = in[i].score;
        }
    }
    for (int c = 0; c < nc; c++) {
        float s = 1.f / (float)cnt[c];
        rr[c].x = round_f((float)sx[4 * c + 0] * s);
        rr[c].y = round_f((float)sx[4 * c + 1] * s);
        rr[c].w = round_f((float)sx[4 * c + 2] * s);
        rr[c].h = round_f((float)sx[4 * c + 3] * s);
        rr[c].score = rw[c];
    }
    int m = 0;
    for (int i = 0; i < nc; i++) {
        const sco_rect *r1 = &rr[i];
        int n1 = cnt[i], j;
        if (n1 <= group_threshold) continue;
        for (j = 0; j < nc; j++) {
            int n2 = cnt[j];
            if (j == i || n2 <= group_threshold) continue;
            const sco_rect *r2 = &rr[j];
            int dx = round_d(r2->w * eps), dy = round_d(r2->h * eps);
            if (r1->x >= r2->x - dx && r1->y >= r2->y - dy && r1->x + r1->w <= r2->x + r2->w + dx &&
                r1->y + r1->h <= r2->y + r2->h + dy && (n2 > (n1 > 3 ? n1 : 3) || n1 < 3))
                break;
        }
        if (j == nc) out[m++] = *r1;
    }
    free(labels);
    free(sx);
    free(cnt);
    free(rlev);
    free(rw);
    free(rr);
    return m;
}

/* The per-image FDDB block (ObjDetector.cpp:228-231): name, count, then
 * "x y w h score" with std::ostream's default double format (%g, 6 digits).
 * Returns the bytes written (excluding the NUL) or the size needed. */
long sco_fddb_format(const char *name, const sco_rect *r, int n, char *buf, long cap) {
    long len = 0;
    char line[128];
    int k;
    long need = (long)strlen(name) + 1;
    need += snprintf(line, sizeof line, "%d\n", n);
    for (k = 0; k < n; k++)
        need += snprintf(line, sizeof line, "%d %d %d %d %g\n", r[k].x, r[k].y, r[k].w, r[k].h,
                         r[k].score);
    if (!buf || cap < need + 1) return need;
    len += sprintf(buf + len, "%s\n%d\n", name, n);
    for (k = 0; k < n; k++)
        len += sprintf(buf + len, "%d %d %d %d %g\n", r[k].x, r[k].y, r[k].w, r[k].h, r[k].score);
    return len;
}
