// sc_jpeg.hpp -- JPEG -> 8-bit gray (cv::imread IMREAD_GRAYSCALE, ObjDetector.cpp:164)
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace sc {
// Decodes `data` to a W x H gray plane (row stride W); out == nullptr only
// reads the header.  Returns 0, or -1 with *err set.
int jpeg_gray(const uint8_t *data, size_t len, std::vector<uint8_t> *out, int *w, int *h,
              std::string *err);
}  // namespace sc
