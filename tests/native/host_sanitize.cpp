// Host-side sanitizer driver ("ASan on the host restatement"): runs
// the product's host translation units -- the in-place .scene/.obj loader and
// the threaded KD build (wr_scene.cpp, the reference's scene.cpp:259-489 and
// KDtreeAccel.cpp:12-307), the threaded verified-BVH build (wr_bvh.cpp), the
// image writers (wr_image.cpp) and the film checkpoint (wr_checkpoint.cpp) --
// on the scenes and malformed inputs named on the command line.  Built by
// tests/test_sanitize.py twice: -fsanitize=address,undefined and
// -fsanitize=thread.  CPU only; no HIP code is compiled in.
//
//   host_sanitize OUTDIR SCENE...     ('!' before a path: the load must fail)
//
// Prints one line per input and "DONE"; any sanitizer report aborts the run
// with a non-zero status (halt_on_error / -fno-sanitize-recover).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "winmad_rt.h"
#include "wr_bvh.h"
#include "wr_scene.h"

static int fail(const std::string& m) {
  std::printf("FAIL %s\n", m.c_str());
  return 1;
}

// the film writers and the checkpoint on a film with every awkward value
static int images_and_checkpoint(const std::string& dir) {
  const int h = 37, w = 53;
  std::vector<float> film(size_t(h) * w * 3);
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> u(-1.f, 4.f);
  for (float& v : film) v = u(rng);
  film[0] = NAN;
  film[1] = INFINITY;
  film[2] = -INFINITY;
  for (const char* ext : {".ppm", ".bmp", ".png", ".pfm"}) {
    const std::string p = dir + "/img" + ext;
    if (wr_film_write_image(film.data(), h, w, 0.5f, 2.2f, 0, p.c_str()) != WR_OK)
      return fail(std::string("write ") + ext + ": " + wr::last_error());
  }
  std::vector<float> sq(size_t(w) * w * 3, 0.25f);
  if (wr_film_write_ppm(sq.data(), w, w, 1.f, 2.2f, 1, (dir + "/sq.ppm").c_str()) != WR_OK)
    return fail("write transposed ppm");
  if (wr_film_write_image(film.data(), h, w, 1.f, 2.2f, 1, (dir + "/bad.ppm").c_str()) == WR_OK)
    return fail("a non-square transpose was accepted");
  if (wr_film_write_image(film.data(), h, w, 1.f, 2.2f, 0, (dir + "/bad.xyz").c_str()) == WR_OK)
    return fail("an unknown extension was accepted");
  const std::string ck = dir + "/ck.bin";
  wr_checkpoint_info info{w, h, WR_CKPT_BDPT, 2, 5, 9, {1u, 2u}};
  if (wr_checkpoint_save(ck.c_str(), &info, film.data()) != WR_OK) return fail("checkpoint save");
  wr_checkpoint_info got{};
  std::vector<float> back(film.size());
  if (wr_checkpoint_load(ck.c_str(), &got, back.data(), static_cast<int64_t>(back.size())) != WR_OK)
    return fail(std::string("checkpoint load: ") + wr::last_error());
  if (std::memcmp(back.data(), film.data(), film.size() * sizeof(float)) != 0) return fail("checkpoint film");
  if (wr_checkpoint_load(ck.c_str(), &got, back.data(), 3) == WR_OK) return fail("short film buffer accepted");
  // truncated and corrupted files
  FILE* f = std::fopen(ck.c_str(), "rb");
  std::vector<unsigned char> raw(1 << 20);
  const size_t n = std::fread(raw.data(), 1, raw.size(), f);
  std::fclose(f);
  for (size_t cut : {size_t(0), size_t(7), size_t(20), size_t(40), n / 2, n - 1}) {
    const std::string t = dir + "/ck_cut.bin";
    FILE* g = std::fopen(t.c_str(), "wb");
    std::fwrite(raw.data(), 1, cut, g);
    std::fclose(g);
    if (wr_checkpoint_load(t.c_str(), &got, back.data(), static_cast<int64_t>(back.size())) == WR_OK)
      return fail("truncated checkpoint accepted at " + std::to_string(cut));
  }
  raw[n / 2] ^= 0x10;
  FILE* g = std::fopen((dir + "/ck_bad.bin").c_str(), "wb");
  std::fwrite(raw.data(), 1, n, g);
  std::fclose(g);
  if (wr_checkpoint_load((dir + "/ck_bad.bin").c_str(), &got, back.data(), static_cast<int64_t>(back.size())) == WR_OK)
    return fail("corrupted checkpoint accepted");
  std::printf("images+checkpoint ok\n");
  return 0;
}

// the same scene through the flat-array path (wr_scene_from_desc's builder)
static int from_arrays(const wr::Scene& s) {
  std::vector<int> type, mat;
  std::vector<float> data, ltri, lle, mats;
  for (const wr::Prim& p : s.prims) {
    type.push_back(p.type);
    mat.push_back(p.mat);
    if (p.type == wr::kTri)
      data.insert(data.end(), {p.p0.x, p.p0.y, p.p0.z, p.p1.x, p.p1.y, p.p1.z, p.p2.x, p.p2.y, p.p2.z});
    else
      data.insert(data.end(), {p.c.x, p.c.y, p.c.z, p.r, 0, 0, 0, 0, 0});
  }
  for (const wr::Light& l : s.lights) {
    const float p1[3] = {l.p0.x + l.d1.x, l.p0.y + l.d1.y, l.p0.z + l.d1.z};
    const float p2[3] = {l.p0.x + l.d2.x, l.p0.y + l.d2.y, l.p0.z + l.d2.z};
    ltri.insert(ltri.end(), {l.p0.x, l.p0.y, l.p0.z, p1[0], p1[1], p1[2], p2[0], p2[1], p2[2]});
    lle.insert(lle.end(), {l.le.x, l.le.y, l.le.z});
  }
  for (const wr::Material& m : s.mats)
    mats.insert(mats.end(), {m.diffuse.x, m.diffuse.y, m.diffuse.z, m.phong.x, m.phong.y, m.phong.z, m.specular.x,
                             m.specular.y, m.specular.z, m.phong_exp, m.index});
  const float pos[3] = {s.cam.pos.x, s.cam.pos.y, s.cam.pos.z}, fwd[3] = {s.cam.fwd.x, s.cam.fwd.y, s.cam.fwd.z},
              up[3] = {s.cam.up.x, s.cam.up.y, s.cam.up.z};
  wr::SceneArrays a{static_cast<int>(s.prims.size()), type.data(), data.data(), mat.data(),
                    static_cast<int>(s.lights.size()), ltri.data(), lle.data(), static_cast<int>(s.mats.size()),
                    mats.data(), pos, fwd, up, s.cam.xres, s.cam.yres, s.cam.fov};
  wr::Scene t;
  std::string err;
  // the result need not equal the loaded scene (lights are rebuilt from their
  // corners): this exercises the builder's memory and threading only
  if (!wr::scene_from_arrays(a, t, err)) std::printf("  from_arrays refused: %s\n", err.c_str());
  // malformed arrays must be refused, not read out of range
  wr::SceneArrays bad = a;
  std::vector<int> badmat(mat);
  if (!badmat.empty()) badmat[0] = -static_cast<int>(s.lights.size()) - 5;  // an emitter id naming no light
  bad.prim_mat = badmat.data();
  wr::Scene u;
  if (!badmat.empty() && wr::scene_from_arrays(bad, u, err)) return fail("emitter matId without a light accepted");
  bad = a;
  bad.n_prims = -1;
  if (wr::scene_from_arrays(bad, u, err)) return fail("negative primitive count accepted");
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return fail("usage: host_sanitize OUTDIR SCENE...");
  const std::string dir = argv[1];
  if (int rc = images_and_checkpoint(dir)) return rc;
  for (int i = 2; i < argc; ++i) {
    const bool must_fail = argv[i][0] == '!';
    const char* path = argv[i] + (must_fail ? 1 : 0);
    wr::Scene s;
    std::string err;
    const bool ok = wr::load_scene(path, s, err);
    if (must_fail) {
      if (ok) return fail(std::string("malformed input accepted: ") + path);
      std::printf("%s refused: %s\n", path, err.c_str());
      continue;
    }
    if (!ok) {
      std::printf("%s: load failed (%s)\n", path, err.c_str());
      continue;  // e.g. a scene whose .obj lines are malformed but the reference would also reject
    }
    const std::string dump = wr::dump_scene(s);
    const uint64_t fp = wr::scene_fingerprint(s);
    wrf::FastHost f;
    if (!s.prims.empty() && !s.lights.empty()) wrf::build_fast(s, f);
    if (int rc = from_arrays(s)) return rc;
    std::printf("%s: %zu prims, %zu kd nodes, dump %zu B, fp %016llx, bvh %s (%zu nodes)\n", path, s.prims.size(),
                s.nodes.size(), dump.size(), static_cast<unsigned long long>(fp), f.ok ? "ok" : f.why.c_str(),
                f.nodes.size());
  }
  std::printf("DONE\n");
  return 0;
}
