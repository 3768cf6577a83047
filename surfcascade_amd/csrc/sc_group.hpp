// sc_group.hpp -- host post-processing (groupRectangles + FDDB block).
#pragma once

#include <string>
#include <vector>

#include "surfcascade.h"

namespace sc {

// cv::groupRectangles(rects, weights = 0s, levelWeights = scores, thr, eps)
std::vector<sc_scored_rect> group_rectangles(const sc_scored_rect *in, int n, int group_threshold,
                                             double eps);
// fast_nms (ObjDetector.cpp:275-383): greedy overlap suppression in the
// reference's own tie order; returns the picked rectangles in pick order.
std::vector<sc_scored_rect> fast_nms(const sc_scored_rect *in, int n, double overlap_th);
// "name\ncount\nx y w h score\n..." (ObjDetector.cpp:228-231)
std::string fddb_block(const char *name, const sc_scored_rect *r, int n);

}  // namespace sc
