// Host-side scene for the MI355X renderer: the reference's Scene::init
// (src/scene/scene.cpp:259-489) -- .scene XML + .obj ingestion, camera
// matrices, area lights, and the SAH KD tree of KDtreeAccel (KDtreeAccel.cpp:12-307)
// -- producing flat arrays that wr_device uploads to HBM.
//
// Float semantics follow the reference statement by statement (this file is
// compiled with -ffp-contract=off) so that triangles, camera matrices and the
// tree are bit-identical to the reference's; tests/test_host.py checks the dump
// against the hash of the reference's own dump.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace wr {

struct F3 {
  float x, y, z;
};

enum PrimType : int { kTri = 0, kSphere = 1 };

struct Prim {
  int type, mat;
  F3 p0, p1, p2;   // triangle vertices (reference objs order)
  F3 c;            // sphere centre
  float r;         // sphere radius
  F3 bl, br;       // AABB after AABB::extend (AABB.h:13-21)
};

struct Light {       // AreaLight (light.h:82-129)
  F3 p0, d1, d2;
  F3 fx, fy, fz;     // localFrame
  F3 le;
  float inv_area;
};

struct Material {    // material.h:7-31
  F3 diffuse, phong, specular;
  float phong_exp, index;
};

struct Camera {      // camera.h:8-27 (+ the two 4x4s the path uses)
  F3 pos, fwd, up;
  float xres, yres, fov, plane_dist;
  float w2r[16], r2w[16];
};

struct KdNode {
  int axis;        // -1 = leaf (KDtreeAccel.cpp:323: axis != -1 means inner)
  float split;
  int right;       // pre-order layout: left child = this + 1
  int first, count;  // leaf: range in refs; inner: count = objNum
};

struct Scene {
  std::vector<Prim> prims;
  std::vector<Light> lights;
  std::vector<Material> mats;
  Camera cam{};
  bool has_camera = false;
  float tot_area = 0.f;
  // KD tree
  int dep_max = 0;
  int max_stack = 0;          // deepest inner-node chain (stack bound for traversal)
  F3 root_l{}, root_r{};
  std::vector<KdNode> nodes;  // pre-order
  std::vector<int> refs;      // leaf primitive indices
  // scene sphere (scene.cpp:483-487)
  F3 sph_c{};
  float sph_r = 0.f, sph_inv_r2 = 0.f;
  int missing_files = 0;      // object files the reference would silently skip
};

// Scene::loadScene(char*) + Scene::init.  Returns false and sets err on a
// malformed file; a missing .obj is silently skipped exactly like the
// reference (tiny_obj_loader.cpp:467-474) and counted in missing_files.
bool load_scene(const char* path, Scene& out, std::string& err);

// The reference's in-memory Scene (scene.h:35-42) as flat arrays
// (wr_scene_desc of include/winmad_rt.h): primitives in objs order, area
// lights, materials, and Camera::setup's arguments.  The KD tree is built
// here, as Scene::init does after loading (scene.cpp:469-489).
struct SceneArrays {
  int n_prims;
  const int* prim_type;    // kTri / kSphere
  const float* prim_data;  // 9 per primitive: p0 p1 p2 | centre, radius
  const int* prim_mat;
  int n_lights;
  const float* light_tri;  // 9 per light: p0 p1 p2
  const float* light_le;   // 3 per light
  int n_materials;
  const float* materials;  // 11 per material: diffuse, phong, specular, phongExp, refracIndex
  const float *cam_pos, *cam_fwd, *cam_up;
  float cam_xres, cam_yres, cam_hfov;
};
bool scene_from_arrays(const SceneArrays& a, Scene& out, std::string& err);

// The reference's tree, built with its exact SAH sweep, event order and
// straddler clipping, but freeing each node's event lists as soon as the
// children own theirs.
void build_kdtree(Scene& s);

// Text dump with the exact format of oracle/ref_driver.cpp `scene`.
std::string dump_scene(const Scene& s);

// 64-bit FNV-1a over what a render reads from the scene: primitives (type,
// material, geometry), lights, materials and the camera.  Checkpoints carry
// it so that a film is never resumed into a render of another scene.
uint64_t scene_fingerprint(const Scene& s);

// Camera::setup (camera.cpp:3-29).
void setup_camera(Camera& c, F3 pos, F3 fwd, F3 up, float xres, float yres, float fov);

// Error message of the last failing wr_* call on this thread (wr_last_error).
int set_error(int code, const std::string& msg);
const char* last_error();

}  // namespace wr
