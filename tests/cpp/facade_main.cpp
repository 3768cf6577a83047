// Drives include/surfcascade.hpp the way ObjDetector.cpp's detect branch would
// (tests/test_facade.py builds and runs it).
//   facade_main MODEL.cfg OUT.cfg            -> Load, print fitted patches, Save
//   facade_main MODEL.cfg OUT.cfg FRAME W H  -> also Detect on a raw u8 frame (GPU)
#include <cstdio>
#include <fstream>
#include <iterator>
#include <vector>

#include "surfcascade.hpp"

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    surfcascade::Model model(argv[1]);
    surfcascade::CascadeClassifier cascade;
    if (model.Load(cascade) != EXIT_SUCCESS) {
        std::fprintf(stderr, "load failed: %s\n", model.last_error.c_str());
        return 1;
    }
    std::vector<std::vector<int>> idx;
    cascade.GetFittedPatchIndexes(idx);
    const auto patches = surfcascade::ExtractPatches(40, 40);
    std::printf("stages %zu patches %zu\n", idx.size(), patches.size());
    for (size_t s = 0; s < idx.size(); s++)
        std::printf("stage %zu theta %.9g weak %zu first_patch %d\n", s,
                    cascade.stage_classifiers[s].theta, idx[s].size(), idx[s][0]);
    surfcascade::Model out(argv[2]);
    if (out.Save(cascade) != EXIT_SUCCESS) return 1;
    if (argc == 4) {  // facade_main MODEL.cfg OUT.cfg IMAGE.jpg: imread + fast_nms (host only)
        const surfcascade::GrayImage g = surfcascade::imread_gray(argv[3]);
        unsigned long sum = 0;
        for (uint8_t v : g.data) sum += v;
        std::printf("image %d %d %lu\n", g.width, g.height, sum);
        std::vector<surfcascade::Rect> r = {{0, 0, 40, 40}, {2, 2, 40, 40}, {100, 100, 40, 40}};
        std::vector<double> s = {0.7, 0.9, 0.8};
        surfcascade::fast_nms(r, s, 0.7);
        for (size_t i = 0; i < r.size(); i++) std::printf("nms %d %d %.3f\n", r[i].x, r[i].y, s[i]);
    }
    if (argc >= 6) {
        std::ifstream f(argv[3], std::ios::binary);
        std::vector<uint8_t> img((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        const int w = std::atoi(argv[4]), h = std::atoi(argv[5]);
        sc_scan_params p = surfcascade::DefaultScanParams();
        p.n_levels = 3;
        surfcascade::Detector det(cascade, p, 0);
        std::vector<surfcascade::Rect> wins;
        std::vector<double> scores;
        det.Detect(img.data(), w, h, w, wins, scores);
        std::printf("detections %zu\n", wins.size());
        for (size_t i = 0; i < wins.size(); i++)
            std::printf("%d %d %d %d %.17g\n", wins[i].x, wins[i].y, wins[i].width, wins[i].height,
                        scores[i]);
        std::vector<int> weights(wins.size(), 0);  // ObjDetector.cpp:223-225
        surfcascade::groupRectangles(wins, weights, scores, 2, 0.2);
        std::printf("%s", surfcascade::FddbBlock("frame", wins, scores).c_str());
        surfcascade::Miner miner(nullptr);  // first round: every stride-10 window
        std::vector<std::vector<std::vector<float>>> negs;
        const bool full = miner.FillNegSamples(img.data(), w, h, w, negs, 5);
        std::printf("mined %zu %d %.9g\n", negs.size(), (int)full, negs.empty() ? 0.0 : negs[4][607][31]);
        // the batch form over [img, img]: the first 5 samples are img's again
        std::vector<std::vector<std::vector<float>>> negs2;
        const std::vector<const uint8_t *> batch = {img.data(), img.data()};
        const bool full2 = miner.FillNegSamples(batch, w, h, w, negs2, 5);
        std::printf("minedb %zu %d %.9g\n", negs2.size(), (int)full2, negs2.empty() ? 0.0 : negs2[4][607][31]);
    }
    return 0;
}
