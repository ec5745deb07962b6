// Film output without OpenCV: ImageFilm::outputImage (src/scene/film.cpp:39-64)
// and the BDPT transpose (bidirPathTracing.cpp:29-46).  The reference hands an
// 8-bit BGR image to cvSaveImage, which picks the file format from the
// extension; the formats here are the ones that need no external library.
//   .ppm  binary P6                  .bmp  24-bit BI_RGB (bottom-up BGR rows)
//   .png  8-bit RGB, stored deflate  .pfm  linear float RGB (scale applied,
//                                          no clamp / gamma: an HDR dump)
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "winmad_rt.h"
#include "wr_scene.h"

namespace {

bool has_ext(const std::string& p, const char* ext) {
  const size_t n = std::strlen(ext);
  if (p.size() < n) return false;
  for (size_t i = 0; i < n; ++i)
    if (std::tolower(static_cast<unsigned char>(p[p.size() - n + i])) != ext[i]) return false;
  return true;
}

// film[i][j] (optionally read transposed) -> scale -> clamp [0,1] -> pow(1/gamma)
// -> (uchar)(x * 255.0), RGB rows top-down (Color3::clamp/gamma/R/G/B, color.h:47-75)
std::vector<uint8_t> to_8bit(const float* film, int h, int w, float scale, float gamma, bool transpose) {
  std::vector<uint8_t> rgb(size_t(h) * w * 3);
  const float inv_gamma = 1.f / gamma;
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) {
      const float* c = transpose ? film + 3 * (size_t(j) * w + i) : film + 3 * (size_t(i) * w + j);
      for (int ch = 0; ch < 3; ++ch) {
        float v = c[ch] * scale;                 // ImageFilm::scale
        v = std::min(1.0f, std::max(v, 0.0f));    // Color3::clamp -> clampVal (math.cpp:3-6), NaN -> 1
        v = std::pow(v, inv_gamma);               // Color3::gamma
        rgb[3 * (size_t(i) * w + j) + ch] = static_cast<uint8_t>(v * 255.0);
      }
    }
  return rgb;
}

void put32le(std::vector<uint8_t>& o, uint32_t v) {
  for (int k = 0; k < 4; ++k) o.push_back(static_cast<uint8_t>(v >> (8 * k)));
}
void put32be(std::vector<uint8_t>& o, uint32_t v) {
  for (int k = 3; k >= 0; --k) o.push_back(static_cast<uint8_t>(v >> (8 * k)));
}

std::vector<uint8_t> bmp(const std::vector<uint8_t>& rgb, int h, int w) {
  const uint32_t row = (3u * w + 3u) & ~3u, data = row * h;
  std::vector<uint8_t> o = {'B', 'M'};
  put32le(o, 54 + data);
  put32le(o, 0);
  put32le(o, 54);
  put32le(o, 40);
  put32le(o, static_cast<uint32_t>(w));
  put32le(o, static_cast<uint32_t>(h));  // positive: bottom-up rows
  o.push_back(1);
  o.push_back(0);  // planes
  o.push_back(24);
  o.push_back(0);  // bits per pixel
  for (int k = 0; k < 6; ++k) put32le(o, k == 1 ? data : 0);  // BI_RGB, size, resolution, palette
  for (int i = h - 1; i >= 0; --i) {
    for (int j = 0; j < w; ++j) {
      const uint8_t* p = &rgb[3 * (size_t(i) * w + j)];
      o.push_back(p[2]);
      o.push_back(p[1]);
      o.push_back(p[0]);
    }
    for (uint32_t k = 3u * w; k < row; ++k) o.push_back(0);
  }
  return o;
}

uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0xffffffffu) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t v = i;
      for (int k = 0; k < 8; ++k) v = (v & 1u) ? 0xedb88320u ^ (v >> 1) : v >> 1;
      table[i] = v;
    }
    init = true;
  }
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xffu] ^ (c >> 8);
  return c;
}

void png_chunk(std::vector<uint8_t>& o, const char* type, const std::vector<uint8_t>& body) {
  put32be(o, static_cast<uint32_t>(body.size()));
  const size_t start = o.size();
  o.insert(o.end(), type, type + 4);
  o.insert(o.end(), body.begin(), body.end());
  put32be(o, crc32(&o[start], o.size() - start) ^ 0xffffffffu);
}

std::vector<uint8_t> png(const std::vector<uint8_t>& rgb, int h, int w) {
  std::vector<uint8_t> raw;  // filter byte 0 + row
  raw.reserve(size_t(h) * (3 * w + 1));
  for (int i = 0; i < h; ++i) {
    raw.push_back(0);
    raw.insert(raw.end(), rgb.begin() + 3 * size_t(i) * w, rgb.begin() + 3 * size_t(i + 1) * w);
  }
  std::vector<uint8_t> z = {0x78, 0x01};  // zlib header, stored deflate blocks
  uint32_t a = 1, b = 0;                  // adler32
  for (uint8_t x : raw) {
    a = (a + x) % 65521u;
    b = (b + a) % 65521u;
  }
  for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
    const size_t n = std::min<size_t>(65535, raw.size() - off);
    const bool last = off + n >= raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back(static_cast<uint8_t>(n));
    z.push_back(static_cast<uint8_t>(n >> 8));
    z.push_back(static_cast<uint8_t>(~n));
    z.push_back(static_cast<uint8_t>(~n >> 8));
    z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
    if (last) break;
  }
  put32be(z, (b << 16) | a);
  std::vector<uint8_t> o = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put32be(ihdr, static_cast<uint32_t>(w));
  put32be(ihdr, static_cast<uint32_t>(h));
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit RGB, deflate, no filter, no interlace
  png_chunk(o, "IHDR", ihdr);
  png_chunk(o, "IDAT", z);
  png_chunk(o, "IEND", {});
  return o;
}

int write_file(const char* path, const std::string& head, const void* data, size_t n) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return wr::set_error(WR_E_IO, std::string("cannot write ") + path);
  const bool ok = std::fwrite(head.data(), 1, head.size(), f) == head.size() && std::fwrite(data, 1, n, f) == n;
  if (std::fclose(f) != 0 || !ok) return wr::set_error(WR_E_IO, std::string("short write to ") + path);
  return WR_OK;
}

}  // namespace

extern "C" {

int wr_film_write_image(const float* film, int height, int width, float scale, float gamma, int transpose,
                        const char* path) {
  if (!film || !path || height <= 0 || width <= 0) return wr::set_error(WR_E_ARG, "bad argument");
  if (transpose && height != width)
    return wr::set_error(WR_E_ARG, "transpose needs a square film (bidirPathTracing.cpp:31-44)");
  const std::string p(path);
  if (has_ext(p, ".pfm")) {  // linear floats, bottom-up rows (PFM convention), little endian
    std::vector<float> out(size_t(height) * width * 3);
    for (int i = 0; i < height; ++i)
      for (int j = 0; j < width; ++j) {
        const float* c = transpose ? film + 3 * (size_t(j) * width + i) : film + 3 * (size_t(i) * width + j);
        for (int ch = 0; ch < 3; ++ch) out[3 * (size_t(height - 1 - i) * width + j) + ch] = c[ch] * scale;
      }
    const std::string head = "PF\n" + std::to_string(width) + " " + std::to_string(height) + "\n-1.0\n";
    return write_file(path, head, out.data(), out.size() * sizeof(float));
  }
  const std::vector<uint8_t> rgb = to_8bit(film, height, width, scale, gamma, transpose != 0);
  if (has_ext(p, ".bmp")) {
    const std::vector<uint8_t> o = bmp(rgb, height, width);
    return write_file(path, "", o.data(), o.size());
  }
  if (has_ext(p, ".png")) {
    const std::vector<uint8_t> o = png(rgb, height, width);
    return write_file(path, "", o.data(), o.size());
  }
  if (has_ext(p, ".ppm") || p.find('.') == std::string::npos) {
    const std::string head = "P6\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
    return write_file(path, head, rgb.data(), rgb.size());
  }
  return wr::set_error(WR_E_ARG, "unsupported image format (use .ppm, .bmp, .png or .pfm): " + p);
}

int wr_film_write_ppm(const float* film, int height, int width, float scale, float gamma, int transpose,
                      const char* path) {
  if (!film || !path || height <= 0 || width <= 0) return wr::set_error(WR_E_ARG, "bad argument");
  if (transpose && height != width)
    return wr::set_error(WR_E_ARG, "transpose needs a square film (bidirPathTracing.cpp:31-44)");
  const std::vector<uint8_t> rgb = to_8bit(film, height, width, scale, gamma, transpose != 0);
  const std::string head = "P6\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
  return write_file(path, head, rgb.data(), rgb.size());
}

}  // extern "C"
