// sc_group.cpp -- post-processing after the detect path (host C++):
// cv::groupRectangles(wins, weights = 0s, levelWeights = scores, 2, 0.2) and
// the FDDB text block (ObjDetector.cpp:223-231).
//
// groupRectangles is OpenCV 3.0.0 objdetect (an external dependency of the
// reference).  Its output is a function of the input rectangles only through
// the connected components of the SimilarRects(eps) graph (a symmetric
// predicate), the per-component integer sums, member counts and maximum
// score, plus the "inside a bigger cluster" filter.  OpenCV finds the
// components with an O(n^2) all-pairs partition; here the pairs come from a
// sweep over x-sorted rectangles (a pair can only be similar when its x
// distance is within eps*(w+h)/2 of either member), then the same union-find.
// Classes are numbered by first appearance in input order, so the output
// order equals OpenCV's for the same input order.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "sc_group.hpp"

namespace sc {

namespace {

// Integer sums and differences of rectangle coordinates in 64 bits: OpenCV
// computes them in int, which gives the same values for every rectangle
// whose coordinates do not overflow (all a detector emits) and undefined
// behaviour otherwise; the 64-bit form is defined for any int32 input
// (tests/test_fuzz_parsers.py runs it under UBSan).
typedef long long i64;

// SimilarRects::operator() (OpenCV cascadedetect.hpp)
inline bool similar(const sc_scored_rect &a, const sc_scored_rect &b, double eps) {
    const double delta = eps * (double)((i64)std::min(a.width, b.width) + std::min(a.height, b.height)) * 0.5;
    return (double)std::llabs((i64)a.x - b.x) <= delta && (double)std::llabs((i64)a.y - b.y) <= delta &&
           (double)std::llabs((i64)a.x + a.width - b.x - b.width) <= delta &&
           (double)std::llabs((i64)a.y + a.height - b.y - b.height) <= delta;
}

struct UnionFind {
    std::vector<int> p, r;
    explicit UnionFind(int n) : p(n), r(n, 0) { std::iota(p.begin(), p.end(), 0); }
    int find(int x) {
        while (p[x] != x) {
            p[x] = p[p[x]];
            x = p[x];
        }
        return x;
    }
    void unite(int a, int b) {
        a = find(a);
        b = find(b);
        if (a == b) return;
        if (r[a] < r[b]) std::swap(a, b);
        p[b] = a;
        if (r[a] == r[b]) r[a]++;
    }
};

}  // namespace

std::vector<sc_scored_rect> group_rectangles(const sc_scored_rect *in, int n, int group_threshold,
                                             double eps) {
    if (group_threshold <= 0 || n <= 0) return std::vector<sc_scored_rect>(in, in + std::max(n, 0));
    // connected components of the similarity graph
    std::vector<int> ord(n);
    std::iota(ord.begin(), ord.end(), 0);
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return in[a].x < in[b].x; });
    UnionFind uf(n);
    for (int s = 0; s < n; s++) {
        const sc_scored_rect &a = in[ord[s]];
        const double reach = eps * (double)((i64)a.width + a.height) * 0.5;  // delta <= this for any partner
        for (int t = s + 1; t < n; t++) {
            const sc_scored_rect &b = in[ord[t]];
            if ((double)((i64)b.x - a.x) > reach) break;
            if (similar(a, b, eps)) uf.unite(ord[s], ord[t]);
        }
    }
    // classes by first appearance (cv::partition's numbering)
    std::vector<int> label(n), cls_of_root(n, -1);
    int nc = 0;
    for (int i = 0; i < n; i++) {
        const int root = uf.find(i);
        if (cls_of_root[root] < 0) cls_of_root[root] = nc++;
        label[i] = cls_of_root[root];
    }
    std::vector<long long> sum((size_t)nc * 4, 0);
    std::vector<int> cnt(nc, 0);
    std::vector<double> best(nc, DBL_MIN);  // rejectWeights init
    for (int i = 0; i < n; i++) {
        const int c = label[i];
        sum[4 * c + 0] += in[i].x;
        sum[4 * c + 1] += in[i].y;
        sum[4 * c + 2] += in[i].width;
        sum[4 * c + 3] += in[i].height;
        cnt[c]++;
        // weights all 0 == rejectLevels: the class keeps its largest levelWeight
        if (in[i].score > best[c]) best[c] = in[i].score;
    }
    // mean rectangle: saturate_cast<int>(sum * (1.f/count)) in f32, ties to even
    std::vector<sc_scored_rect> rr(nc);
    for (int c = 0; c < nc; c++) {
        const float s = 1.f / (float)cnt[c];
        rr[c].x = (int)std::lrintf((float)sum[4 * c + 0] * s);
        rr[c].y = (int)std::lrintf((float)sum[4 * c + 1] * s);
        rr[c].width = (int)std::lrintf((float)sum[4 * c + 2] * s);
        rr[c].height = (int)std::lrintf((float)sum[4 * c + 3] * s);
        rr[c].score = best[c];
    }
    std::vector<sc_scored_rect> out;
    for (int i = 0; i < nc; i++) {
        const int n1 = cnt[i];
        if (n1 <= group_threshold) continue;  // too few similar rectangles
        const sc_scored_rect &r1 = rr[i];
        bool inside = false;  // a small rectangle inside a better-supported large one
        for (int j = 0; j < nc && !inside; j++) {
            const int n2 = cnt[j];
            if (j == i || n2 <= group_threshold) continue;
            const sc_scored_rect &r2 = rr[j];
            const i64 dx = (int)std::lrint(r2.width * eps), dy = (int)std::lrint(r2.height * eps);
            inside = r1.x >= r2.x - dx && r1.y >= r2.y - dy &&
                     (i64)r1.x + r1.width <= (i64)r2.x + r2.width + dx &&
                     (i64)r1.y + r1.height <= (i64)r2.y + r2.height + dy && (n2 > std::max(3, n1) || n1 < 3);
        }
        if (!inside) out.push_back(r1);
    }
    return out;
}

std::string fddb_block(const char *name, const sc_scored_rect *r, int n) {
    std::string s(name);
    s += '\n';
    char line[160];
    std::snprintf(line, sizeof line, "%d\n", n);
    s += line;
    for (int k = 0; k < n; k++) {  // std::ostream's default double format: %g
        std::snprintf(line, sizeof line, "%d %d %d %d %g\n", r[k].x, r[k].y, r[k].width,
                      r[k].height, r[k].score);
        s += line;
    }
    return s;
}

// fast_nms (ObjDetector.cpp:318-383; commented out at :223, the reference's
// alternative to groupRectangles).  Followed literally, including its
// quirks: sort_idx (:275-288) is an exchange sort ASCENDING by score (despite
// its comment) whose tie order depends on the swaps, so it is simulated as
// written, O(n^2); the pick is the LAST remaining index (the best score);
// overlap uses +1 areas, a float inverse area 1.0f/((w+1)*(h+1)) and the
// int*float product compared with the double threshold; suppressed entries
// are compacted by sort_stable (:290-313).
std::vector<sc_scored_rect> fast_nms(const sc_scored_rect *in, int n, double overlap_th) {
    std::vector<int> idx(std::max(n, 0));
    std::vector<float> inv(std::max(n, 0));
    std::iota(idx.begin(), idx.end(), 0);
    for (int i = 0; i < n; i++)  // sort_idx
        for (int j = i + 1; j < n; j++) {
            const int ti = idx[i], tj = idx[j];
            if (in[tj].score < in[ti].score) {
                idx[i] = tj;
                idx[j] = ti;
            }
        }
    for (int i = 0; i < n; i++) {
        const sc_scored_rect &r = in[idx[i]];
        inv[idx[i]] = 1.0f / (float)(((i64)r.width + 1) * ((i64)r.height + 1));
    }
    auto sort_stable = [&](int cnt) {  // :290-313, returns the new count
        int i = 0, j = 0;
        while (i < cnt) {
            if (idx[i] == -1) {
                if (j < i + 1) j = i + 1;
                while (j < cnt) {
                    if (idx[j] == -1) {
                        ++j;
                    } else {
                        idx[i] = idx[j];
                        idx[j] = -1;
                        j++;
                        break;
                    }
                }
                if (j == cnt) return i;
            }
            ++i;
        }
        return i;
    };
    std::vector<sc_scored_rect> picked;
    int count = n;
    while (count > 0) {
        const int tmp = count - 1, last = idx[tmp];
        picked.push_back(in[last]);
        const i64 x0 = in[last].x, y0 = in[last].y;
        const i64 x1 = x0 + in[last].width, y1 = y0 + in[last].height;
        idx[tmp] = -1;
        for (int i = tmp - 1; i != -1; i--) {
            const sc_scored_rect &r = in[idx[i]];
            i64 tx0 = std::max<i64>(x0, r.x), ty0 = std::max<i64>(y0, r.y);
            const i64 tx1 = std::min<i64>(x1, (i64)r.x + r.width), ty1 = std::min<i64>(y1, (i64)r.y + r.height);
            tx0 = tx1 - tx0 + 1;
            ty0 = ty1 - ty0 + 1;
            if (tx0 > 0 && ty0 > 0 && (double)((float)((double)tx0 * (double)ty0) * inv[idx[i]]) > overlap_th)
                idx[i] = -1;
        }
        count = sort_stable(count);
    }
    return picked;
}

}  // namespace sc
