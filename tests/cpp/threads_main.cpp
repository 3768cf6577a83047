// Two threads, two detectors, one library: the C ABI's thread-safety promise
// (surfcascade.h: distinct detectors may be used from different threads; the
// error message is thread-local).  Built against the ThreadSanitizer build of
// the host code by tests/test_threads.py; any TSan report fails the test.
//
//   threads_main CFG FRAMES W H N [JPEG]
// CFG: model file; FRAMES: N raw u8 frames of W x H back to back.
// Each thread parses + saves the model, groups rectangles, runs fast_nms,
// decodes the JPEG, provokes its own error, and -- when a GPU is present --
// creates its own detector on device 0 and detects every frame R times,
// comparing with the main thread's single-threaded result.
// Prints "ok detect=<0|1>" on success.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "surfcascade.h"

namespace {

std::string slurp(const char *path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

struct Result {
    std::vector<sc_window> wins;
    std::vector<int> counts;
};

bool same(const Result &a, const Result &b) {
    if (a.counts != b.counts || a.wins.size() != b.wins.size()) return false;
    for (size_t i = 0; i < a.wins.size(); i++)
        if (std::memcmp(&a.wins[i], &b.wins[i], sizeof(sc_window)) != 0) return false;
    return true;
}

int detect_all(sc_detector *d, const std::vector<const uint8_t *> &frames, int w, int h, Result &r) {
    r.counts.assign(frames.size(), 0);
    r.wins.resize(1 << 16);
    int st = sc_detect_batch(d, frames.data(), (int)frames.size(), w, h, w, r.wins.data(), (int)r.wins.size(),
                             r.counts.data());
    if (st != SC_OK) return st;
    size_t n = 0;
    for (int c : r.counts) n += (size_t)c;
    r.wins.resize(n);
    return SC_OK;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s CFG FRAMES W H N [JPEG]\n", argv[0]);
        return 2;
    }
    const std::string cfg = slurp(argv[1]);
    const std::string raw = slurp(argv[2]);
    const int w = std::atoi(argv[3]), h = std::atoi(argv[4]), n = std::atoi(argv[5]);
    const std::string jpeg = argc > 6 ? slurp(argv[6]) : std::string();
    if ((long long)raw.size() != (long long)w * h * n) {
        std::fprintf(stderr, "frame file size\n");
        return 2;
    }
    std::vector<const uint8_t *> frames;
    for (int f = 0; f < n; f++) frames.push_back(reinterpret_cast<const uint8_t *>(raw.data()) + (size_t)f * w * h);
    sc_scan_params prm;
    sc_scan_params_default(&prm);
    prm.n_levels = 4;

    sc_model *m0 = nullptr;
    if (sc_model_parse(cfg.data(), cfg.size(), &m0) != SC_OK) {
        std::fprintf(stderr, "parse: %s\n", sc_last_error());
        return 1;
    }
    // the single-threaded result (or no device at all)
    Result ref;
    bool have_gpu = false;
    {
        sc_detector *d = nullptr;
        const int st = sc_detector_create_from_model(m0, &prm, 0, &d);
        if (st == SC_OK) {
            have_gpu = true;
            if (detect_all(d, frames, w, h, ref) != SC_OK) {
                std::fprintf(stderr, "detect: %s\n", sc_last_error());
                return 1;
            }
            sc_detector_destroy(d);
        } else if (st != SC_ERR_DEVICE) {
            std::fprintf(stderr, "create: %s\n", sc_last_error());
            return 1;
        }
    }
    // rectangles for the post-processing calls
    std::vector<sc_scored_rect> rects;
    for (int i = 0; i < 400; i++)
        rects.push_back(sc_scored_rect{(i * 37) % 300, (i * 53) % 200, 40 + i % 7, 40 + i % 7, 0.5 + (i % 13) * 0.01});

    std::atomic<int> failures{0};
    auto worker = [&](int id) {
        const std::string path = std::string(argv[2]) + ".t" + std::to_string(id) + ".cfg";
        sc_detector *d = nullptr;
        if (have_gpu && sc_detector_create_from_model(m0, &prm, 0, &d) != SC_OK) failures++;
        for (int it = 0; it < 3; it++) {
            sc_model *m = nullptr;
            if (sc_model_parse(cfg.data(), cfg.size(), &m) != SC_OK || sc_model_save(m, path.c_str()) != SC_OK)
                failures++;
            sc_model_free(m);
            if (slurp(path.c_str()) != cfg) failures++;
            std::vector<sc_scored_rect> out(rects.size());
            int no = 0;
            if (sc_group_rectangles(rects.data(), (int)rects.size(), 2, 0.2, out.data(), (int)out.size(), &no) != SC_OK)
                failures++;
            if (sc_fast_nms(rects.data(), (int)rects.size(), 0.3, out.data(), (int)out.size(), &no) != SC_OK)
                failures++;
            if (!jpeg.empty()) {
                int jw = 0, jh = 0;
                std::vector<uint8_t> g(1 << 22);
                if (sc_decode_jpeg_gray(reinterpret_cast<const uint8_t *>(jpeg.data()), jpeg.size(), g.data(),
                                        g.size(), &jw, &jh) != SC_OK)
                    failures++;
            }
            // this thread's error message stays its own
            const std::string bad = "stages = ( " + std::to_string(id);
            sc_model *mb = nullptr;
            if (sc_model_parse(bad.data(), bad.size(), &mb) == SC_OK) failures++;
            const std::string e1 = sc_last_error();
            std::this_thread::yield();
            if (e1.empty() || e1 != sc_last_error()) failures++;
            if (d) {
                Result r;
                if (detect_all(d, frames, w, h, r) != SC_OK || !same(r, ref)) failures++;
            }
        }
        if (d) sc_detector_destroy(d);
        std::remove(path.c_str());
    };
    std::thread t0(worker, 0), t1(worker, 1);
    t0.join();
    t1.join();
    sc_model_free(m0);
    if (failures.load()) {
        std::fprintf(stderr, "%d failures\n", failures.load());
        return 1;
    }
    std::printf("ok detect=%d detections=%zu\n", have_gpu ? 1 : 0, ref.wins.size());
    return 0;
}
