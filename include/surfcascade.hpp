// surfcascade.hpp -- header-only C++ facade over the C ABI (surfcascade.h),
// shaped like the reference's in-process API so the detect branch of
// ObjDetector.cpp can switch with minimal edits:
//
//   reference                                   here
//   Model(string) / Load / Save (Model.h:15-18) surfcascade::Model
//   CascadeClassifier::stage_classifiers,       surfcascade::CascadeClassifier
//     GetFittedPatchIndexes (CascadeClassifier.h:28-32)
//   StageClassifier::theta (StageClassifier.h:24), surfcascade::StageClassifier
//   LogisticRegression::{patch_index, w}         surfcascade::LogisticRegression
//   DenseSURFFeatureExtractor::ExtractPatches    surfcascade::ExtractPatches
//   the scan loop ObjDetector.cpp:160-220        surfcascade::Detector::Detect
//
// Errors: Load/Save return EXIT_SUCCESS / EXIT_FAILURE like the reference
// (message in Model::last_error); Detector throws surfcascade::Error.
#ifndef SURFCASCADE_HPP
#define SURFCASCADE_HPP

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "surfcascade.h"

namespace surfcascade {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc) {
    if (rc < 0) throw Error(rc, sc_last_error());
}

struct Rect {
    int x, y, width, height;
};

struct LogisticRegression {
    int patch_index = 0;
    std::vector<float> w;  // 33
    double bias = 1.0;
};

struct StageClassifier {
    float theta = 0.0f;
    std::vector<LogisticRegression> weak_classifiers;
    void GetFittedPatchIndexes(std::vector<int> &idx) const {
        for (const auto &wk : weak_classifiers) idx.push_back(wk.patch_index);
    }
};

class CascadeClassifier {
   public:
    std::vector<StageClassifier> stage_classifiers;

    void GetFittedPatchIndexes(std::vector<std::vector<int>> &patch_indexes) const {
        for (const auto &s : stage_classifiers) {
            std::vector<int> v;
            s.GetFittedPatchIndexes(v);
            patch_indexes.push_back(v);
        }
    }
    const sc_model *handle() const { return model_.get(); }

   private:
    friend class Model;
    struct Free {
        void operator()(sc_model *m) const { sc_model_free(m); }
    };
    std::shared_ptr<sc_model> model_;
    void adopt(sc_model *m) {
        model_.reset(m, Free());
        stage_classifiers.clear();
        for (int s = 0; s < sc_model_num_stages(m); s++) {
            StageClassifier st;
            int nw = 0;
            check(sc_model_stage(m, s, &st.theta, &nw));
            for (int k = 0; k < nw; k++) {
                LogisticRegression wk;
                wk.w.resize(33);
                check(sc_model_weak(m, s, k, &wk.patch_index, wk.w.data(), &wk.bias));
                st.weak_classifiers.push_back(wk);
            }
            stage_classifiers.push_back(st);
        }
    }
};

class Model {
   public:
    std::string model_cfg, last_error;
    explicit Model(std::string cfg) : model_cfg(std::move(cfg)) {}

    int Load(CascadeClassifier &c) {
        sc_model *m = nullptr;
        if (sc_model_load(model_cfg.c_str(), &m) != SC_OK) {
            last_error = sc_last_error();
            return EXIT_FAILURE;
        }
        c.adopt(m);
        return EXIT_SUCCESS;
    }
    int Save(const CascadeClassifier &c) {
        if (!c.handle() || sc_model_save(c.handle(), model_cfg.c_str()) != SC_OK) {
            last_error = c.handle() ? sc_last_error() : "cascade not loaded";
            return EXIT_FAILURE;
        }
        return EXIT_SUCCESS;
    }
};

inline std::vector<Rect> ExtractPatches(int tmpl_w = 40, int tmpl_h = 40) {
    int n = sc_extract_patches(tmpl_w, tmpl_h, nullptr, 0);
    check(n);
    std::vector<int32_t> r((size_t)n * 4);
    sc_extract_patches(tmpl_w, tmpl_h, r.data(), n);
    std::vector<Rect> out(n);
    for (int i = 0; i < n; i++) out[i] = {r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]};
    return out;
}

// cv::groupRectangles(rectList, weights, levelWeights, groupThreshold, eps)
// as ObjDetector.cpp:224-225 calls it (weights all 0, levelWeights = scores):
// rectList becomes the cluster means, levelWeights their best scores and
// weights 0 per output rectangle.
inline void groupRectangles(std::vector<Rect> &rectList, std::vector<int> &weights,
                            std::vector<double> &levelWeights, int groupThreshold,
                            double eps = 0.2) {
    if (levelWeights.size() != rectList.size()) throw Error(SC_ERR_INVALID, "levelWeights size");
    std::vector<sc_scored_rect> in(rectList.size()), out(rectList.size() + 1);
    for (size_t i = 0; i < rectList.size(); i++)
        in[i] = {rectList[i].x, rectList[i].y, rectList[i].width, rectList[i].height,
                 levelWeights[i]};
    int n = 0;
    check(sc_group_rectangles(in.data(), (int)in.size(), groupThreshold, eps, out.data(),
                              (int)out.size(), &n));
    rectList.clear();
    levelWeights.clear();
    for (int i = 0; i < n; i++) {
        rectList.push_back({out[i].x, out[i].y, out[i].width, out[i].height});
        levelWeights.push_back(out[i].score);
    }
    weights.assign(n, 0);
}

// fast_nms(rects, scores, overlap_th) (ObjDetector.cpp:318-383): rects and
// scores become the picked windows, best first.
inline void fast_nms(std::vector<Rect> &rects, std::vector<double> &scores, double overlap_th) {
    if (scores.size() != rects.size()) throw Error(SC_ERR_INVALID, "scores size");
    std::vector<sc_scored_rect> in(rects.size()), out(rects.size() + 1);
    for (size_t i = 0; i < rects.size(); i++)
        in[i] = {rects[i].x, rects[i].y, rects[i].width, rects[i].height, scores[i]};
    int n = 0;
    check(sc_fast_nms(in.data(), (int)in.size(), overlap_th, out.data(), (int)out.size(), &n));
    rects.clear();
    scores.clear();
    for (int i = 0; i < n; i++) {
        rects.push_back({out[i].x, out[i].y, out[i].width, out[i].height});
        scores.push_back(out[i].score);
    }
}

// A gray image as cv::imread(path, cv::IMREAD_GRAYSCALE) returns it for a
// JPEG file (ObjDetector.cpp:164): continuous rows, stride = width.
struct GrayImage {
    int width = 0, height = 0;
    std::vector<uint8_t> data;
    bool empty() const { return data.empty(); }
};
inline GrayImage imread_gray(const std::string &path) {
    GrayImage g;
    int rc = sc_imread_gray(path.c_str(), nullptr, 0, &g.width, &g.height);
    if (rc != SC_ERR_CAPACITY) check(rc);
    g.data.resize((size_t)g.width * g.height);
    check(sc_imread_gray(path.c_str(), g.data.data(), g.data.size(), &g.width, &g.height));
    return g;
}

// The per-image block of the reference's output file (ObjDetector.cpp:228-231).
inline std::string FddbBlock(const std::string &name, const std::vector<Rect> &wins,
                             const std::vector<double> &scores) {
    std::vector<sc_scored_rect> r(wins.size());
    for (size_t i = 0; i < wins.size(); i++)
        r[i] = {wins[i].x, wins[i].y, wins[i].width, wins[i].height, scores[i]};
    size_t len = 0;
    int rc = sc_fddb_format(name.c_str(), r.data(), (int)r.size(), nullptr, 0, &len);
    if (rc != SC_ERR_CAPACITY) check(rc);
    std::string s(len + 1, '\0');
    check(sc_fddb_format(name.c_str(), r.data(), (int)r.size(), &s[0], s.size(), &len));
    s.resize(len);
    return s;
}

inline sc_scan_params DefaultScanParams() {
    sc_scan_params p;
    sc_scan_params_default(&p);
    return p;
}

// One GPU's detector (device model + buffers + one HIP stream).
class Detector {
   public:
    Detector(const CascadeClassifier &c, const sc_scan_params &p = DefaultScanParams(),
             int device = 0) {
        sc_detector *d = nullptr;
        check(sc_detector_create_from_model(c.handle(), &p, device, &d));
        det_.reset(d);
    }
    // The reference's per-image scan (ObjDetector.cpp:165-220): raw windows
    // (before groupRectangles) and their scores, sorted by (level, y, x).
    void Detect(const uint8_t *gray, int w, int h, int stride, std::vector<Rect> &wins,
                std::vector<double> &scores) {
        std::vector<sc_window> out(1024);
        int n = 0;
        int rc = sc_detect(det_.get(), gray, w, h, stride, out.data(), (int)out.size(), &n);
        if (rc == SC_ERR_CAPACITY) {
            out.resize(n);
            rc = sc_detect(det_.get(), gray, w, h, stride, out.data(), (int)out.size(), &n);
        }
        check(rc);
        wins.clear();
        scores.clear();
        for (int i = 0; i < n; i++) {
            wins.push_back({out[i].x, out[i].y, out[i].w, out[i].h});
            scores.push_back(out[i].score);
        }
    }
    sc_detector *handle() { return det_.get(); }

   private:
    struct Free {
        void operator()(sc_detector *d) const { sc_detector_destroy(d); }
    };
    std::unique_ptr<sc_detector, Free> det_;
};

// Hard-negative mining (DenseSURFFeatureExtractor::FillNegSamples,
// DenseSURFFeatureExtractor.cpp:124-195) on the GPU: cascade == nullptr is
// the first round (every stride-10 window is a candidate).
class Miner {
   public:
    explicit Miner(const CascadeClassifier *cascade, int tmpl_w = 40, int tmpl_h = 40,
                   int device = 0)
        : n_patches_(sc_extract_patches(tmpl_w, tmpl_h, nullptr, 0)) {
        sc_detector *d = nullptr;
        check(sc_miner_create(cascade ? cascade->handle() : nullptr, tmpl_w, tmpl_h, device, &d));
        det_.reset(d);
    }
    // One negative image: appends the descriptors (features_img: n_patches x
    // 32, as ExtractFeatures fills it) of its candidates, in (level, y, x)
    // order, until features_all holds n_total samples; true once it does.
    bool FillNegSamples(const uint8_t *gray, int w, int h, int stride,
                        std::vector<std::vector<std::vector<float>>> &features_all, size_t n_total) {
        if (features_all.size() >= n_total) return true;
        const int want = (int)(n_total - features_all.size());
        std::vector<sc_window> wins(want);
        std::vector<float> feat((size_t)want * n_patches_ * 32);
        int n = 0;
        const int rc = sc_mine(det_.get(), gray, w, h, stride, wins.data(), feat.data(), want, &n);
        if (rc != SC_ERR_CAPACITY) check(rc);
        const int kept = std::min(n, want);
        for (int i = 0; i < kept; i++) {
            std::vector<std::vector<float>> sample(n_patches_);
            for (int j = 0; j < n_patches_; j++) {
                const float *f = &feat[((size_t)i * n_patches_ + j) * 32];
                sample[j].assign(f, f + 32);
            }
            features_all.push_back(std::move(sample));
        }
        return features_all.size() >= n_total;
    }
    // The same over several negative images of one size in one pass
    // (sc_mine_batch): the loop of :132-190 over a chunk of the image list.
    bool FillNegSamples(const std::vector<const uint8_t *> &grays, int w, int h, int stride,
                        std::vector<std::vector<std::vector<float>>> &features_all, size_t n_total) {
        if (features_all.size() >= n_total || grays.empty()) return features_all.size() >= n_total;
        const int want = (int)(n_total - features_all.size());
        std::vector<sc_window> wins(want);
        std::vector<float> feat((size_t)want * n_patches_ * 32);
        std::vector<int> counts(grays.size());
        const int rc = sc_mine_batch(det_.get(), grays.data(), (int)grays.size(), w, h, stride, wins.data(),
                                     feat.data(), want, counts.data());
        if (rc != SC_ERR_CAPACITY) check(rc);
        long long total = 0;
        for (int c : counts) total += c;
        const int kept = (int)std::min<long long>(total, want);
        for (int i = 0; i < kept; i++) {
            std::vector<std::vector<float>> sample(n_patches_);
            for (int j = 0; j < n_patches_; j++) {
                const float *f = &feat[((size_t)i * n_patches_ + j) * 32];
                sample[j].assign(f, f + 32);
            }
            features_all.push_back(std::move(sample));
        }
        return features_all.size() >= n_total;
    }

   private:
    struct Free {
        void operator()(sc_detector *d) const { sc_detector_destroy(d); }
    };
    int n_patches_;
    std::unique_ptr<sc_detector, Free> det_;
};

}  // namespace surfcascade

#endif  // SURFCASCADE_HPP
