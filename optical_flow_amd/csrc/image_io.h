// Host image I/O shared by the data path (SURVEY.md §8 f row 1: data_reader.py) and the flow
// visualisation (row 4: drawing.py).  PNG only: KITTI raw frames are 8-bit RGB PNGs.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace oflow {
namespace png {

struct Info {
  int w = 0, h = 0;
  int depth = 0;      // bits per sample: 1, 2, 4, 8, 16
  int ctype = 0;      // 0 gray, 2 RGB, 3 palette, 4 gray+alpha, 6 RGBA
  int interlace = 0;  // 0 none, 1 Adam7
  int channels() const { return ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 6 ? 4 : 1; }
};

// Header of a PNG file held in memory (reads the signature and IHDR only).
bool parse_info(const uint8_t* data, size_t n, Info& info, std::string& err);
// Read a whole file into `buf`.
bool read_file(const char* path, std::vector<uint8_t>& buf, std::string& err);
// Read only the first bytes of a file (signature + IHDR) and parse them.
bool file_info(const char* path, Info& info, std::string& err);
// Decode to 8-bit BGR, h x w x 3 interleaved, the array cv2.imread(path) returns with its
// default IMREAD_COLOR flag (data_reader.py:53-54).  `out` holds at least h*w*3 bytes.
bool decode_bgr(const uint8_t* data, size_t n, uint8_t* out, size_t cap, Info& info,
                std::string& err);
// Encode an 8-bit image (c = 1 gray, 3 BGR, 4 BGRA; stored as gray / RGB / RGBA).
// filter: 0-4 = that PNG filter on every row, 5 = per-row minimum-sum-of-|residual|
// heuristic, 6 = cycle 0..4 by row (decoder coverage).  level: zlib level 0-9.
bool encode(const uint8_t* img, int h, int w, int c, int filter, int level,
            std::vector<uint8_t>& out, std::string& err);

}  // namespace png
}  // namespace oflow
