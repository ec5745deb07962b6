// Film checkpoint / resume.  The reference keeps its film only in
// memory while BidirPathTracing::render loops over iterations
// (bidirPathTracing.cpp:23-27); an interrupted render is lost.  Iterations
// (and PT samples) are independent and keyed by their global index (counter
// RNG), so a render resumes exactly by loading the accumulated film and
// rendering the remaining indices with iter_begin = done.
//
// File: "WRCKPT01" | wr_checkpoint_info (32 bytes) | FNV-1a 64 of the film
// bytes | height x width x 3 float32 (the accumulated, unscaled film).
// Written to <path>.tmp and renamed over <path>, so a crash mid-write leaves
// the previous checkpoint intact.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "winmad_rt.h"
#include "wr_scene.h"

namespace {
constexpr char kMagic[8] = {'W', 'R', 'C', 'K', 'P', 'T', '0', '1'};
static_assert(sizeof(wr_checkpoint_info) == 32, "checkpoint header layout");

uint64_t fnv1a(const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}
bool valid(const wr_checkpoint_info& i) {
  return i.width > 0 && i.height > 0 && i.kind >= WR_CKPT_BDPT && i.kind <= WR_CKPT_PT && i.done >= 0 &&
         i.total >= i.done && static_cast<int64_t>(i.width) * i.height < (int64_t(1) << 31) / 3;
}
}  // namespace

extern "C" {

int wr_checkpoint_save(const char* path, const wr_checkpoint_info* info, const float* film) {
  if (!path || !info || !film) return wr::set_error(WR_E_ARG, "null argument");
  if (!valid(*info)) return wr::set_error(WR_E_ARG, "bad checkpoint header (size, kind or done > total)");
  const size_t nf = size_t(info->width) * info->height * 3;
  const uint64_t h = fnv1a(film, nf * sizeof(float));
  const std::string tmp = std::string(path) + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return wr::set_error(WR_E_IO, "cannot write " + tmp);
  bool ok = std::fwrite(kMagic, 1, 8, f) == 8 && std::fwrite(info, sizeof *info, 1, f) == 1 &&
            std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(film, sizeof(float), nf, f) == nf;
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path) != 0) {
    std::remove(tmp.c_str());
    return wr::set_error(WR_E_IO, std::string("cannot write checkpoint ") + path);
  }
  return WR_OK;
}

int wr_checkpoint_load(const char* path, wr_checkpoint_info* info, float* film, int64_t film_floats) {
  if (!path || !info) return wr::set_error(WR_E_ARG, "null argument");
  FILE* f = std::fopen(path, "rb");
  if (!f) return wr::set_error(WR_E_IO, std::string("cannot open checkpoint ") + path);
  char magic[8];
  wr_checkpoint_info hd;
  uint64_t h = 0;
  const bool head = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kMagic, 8) == 0 &&
                    std::fread(&hd, sizeof hd, 1, f) == 1 && std::fread(&h, sizeof h, 1, f) == 1 && valid(hd);
  if (!head) {
    std::fclose(f);
    return wr::set_error(WR_E_IO, std::string("not a winmad_rt checkpoint: ") + path);
  }
  *info = hd;
  if (!film) {  // header only
    std::fclose(f);
    return WR_OK;
  }
  const size_t nf = size_t(hd.width) * hd.height * 3;
  if (film_floats != static_cast<int64_t>(nf)) {
    std::fclose(f);
    return wr::set_error(WR_E_ARG, "film buffer size does not match the checkpoint (" + std::to_string(nf) +
                                       " floats)");
  }
  const bool body = std::fread(film, sizeof(float), nf, f) == nf;
  std::fclose(f);
  if (!body || fnv1a(film, nf * sizeof(float)) != h)
    return wr::set_error(WR_E_IO, std::string("checkpoint truncated or corrupt: ") + path);
  return WR_OK;
}

}  // extern "C"
