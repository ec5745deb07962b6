// Test infrastructure only: a driver main() linked against the reference's own
// translation units (compiled from /root/reference by oracle/Makefile into
// oracle/_ref/).  It calls the reference's public API and prints golden vectors
// in hex-float text so tests/golden/ fixtures can pin oracle/cpuref.c and the
// HIP path.  Nothing here re-implements reference behaviour.
//
//   refdrv mt     SEED N                         MT19937 randUInt stream (rng.cpp:24-62)
//   refdrv scene  SCENE PARA                     loader + camera + KD tree dump (scene.cpp:259-489,
//                                                KDtreeAccel.cpp:12-307)
//   refdrv rays   SCENE PARA CORPUS.f32          Scene::intersect / occluded per ray (scene.cpp:21-81)
//   refdrv kat    SCENE PARA N SEED              BSDF / AreaLight / sampler / camera known answers
//   refdrv bdpt   SCENE PARA ITERS SEED OUT.f32  BidirPathTracing::render, film pre-transpose
//   refdrv pt     SCENE PARA SEED OUT.f32        PathIntegrator via SurfaceIntegrator::render
//   refdrv vcm    SCENE PARA ITERS SEED OUT.f32  VertexCM::render (ref_driver_vcm.cpp)
//   refdrv image  H W ITERS TRANSPOSE IN.f32 OUT.rgb
//                 the 8-bit pixels ImageFilm::outputImage hands to cvSaveImage
//                 (film.cpp:39-64): a float film (H x W x 3) -> [transpose, as
//                 BidirPathTracing/VertexCM::outputImage do first,
//                 bidirPathTracing.cpp:31-41] -> ImageFilm::scale(1.f / ITERS)
//                 -> clamp -> gamma(2.2) -> Color3::R/G/B (color.h:47-75),
//                 written as RGB rows (the reference stores B, G, R per pixel)
//
// Every command chdir()s to $REFDRV_CWD (if set) after static initialisation so the
// reference's debug files (bidirPathTracing.cpp:3, vertexcm.h:10) land in a scratch directory.
#include "surfaceIntegrator/bidirPathTracing.h"
#include "surfaceIntegrator/pathIntegrator.h"
#include "material/fresnel.h"
#include <map>
#include <ctime>
#include <cstdlib>
#include <unistd.h>

static std::map<const Geometry*, int> g_index;
int refdrv_vcm(int argc, char** argv, Parameters& para);  // ref_driver_vcm.cpp

static void hv(FILE* f, float x) { fprintf(f, " %a", (double)x); }
static void hv3(FILE* f, const Vector3& v) { hv(f, v.x); hv(f, v.y); hv(f, v.z); }
static void hc3(FILE* f, const Color3& c) { hv(f, c.r); hv(f, c.g); hv(f, c.b); }

static void index_objs(Scene& s) {
    g_index.clear();
    for (size_t i = 0; i < s.objs.size(); i++) g_index[s.objs[i]] = (int)i;
}

static void dump_tree(FILE* f, KDtreeAccelNode* tr) {
    if (!tr) return;
    if (tr->axis == -1) {  // leaf exactly as traverse() decides (KDtreeAccel.cpp:323-324)
        fprintf(f, "L %d", tr->objNum);
        for (int i = 0; i < tr->objNum; i++) fprintf(f, " %d", g_index[tr->objlist[i]]);
        fprintf(f, "\n");
        return;
    }
    fprintf(f, "I %d", tr->axis);
    hv(f, tr->splitPlane);
    fprintf(f, " %d\n", tr->objNum);
    dump_tree(f, tr->left);
    dump_tree(f, tr->right);
}

static void cmd_scene(Scene& s) {
    FILE* f = stdout;
    fprintf(f, "nobjs %d\n", (int)s.objs.size());
    for (size_t i = 0; i < s.objs.size(); i++) {
        Triangle* t = dynamic_cast<Triangle*>(s.objs[i]);
        Sphere* sp = dynamic_cast<Sphere*>(s.objs[i]);
        if (t) { fprintf(f, "tri %d", t->matId); hv3(f, t->p0); hv3(f, t->p1); hv3(f, t->p2); }
        else { fprintf(f, "sph %d", sp->matId); hv3(f, sp->center); hv(f, sp->radius); }
        fprintf(f, "\n");
    }
    fprintf(f, "nlights %d\n", (int)s.lights.size());
    for (size_t i = 0; i < s.lights.size(); i++) {
        AreaLight* l = dynamic_cast<AreaLight*>(s.lights[i]);
        fprintf(f, "light");
        hv3(f, l->p0); hv3(f, l->d1); hv3(f, l->d2);
        hv3(f, l->localFrame.x); hv3(f, l->localFrame.y); hv3(f, l->localFrame.z);
        hc3(f, l->intensity); hv(f, l->invArea);
        fprintf(f, "\n");
    }
    fprintf(f, "nmat %d\n", (int)s.materials.size());
    for (size_t i = 0; i < s.materials.size(); i++) {
        const Material& m = s.materials[i];
        fprintf(f, "mat"); hc3(f, m.diffuse); hc3(f, m.phong); hv(f, m.phongExp);
        hc3(f, m.specular); hv(f, m.index); fprintf(f, "\n");
    }
    Camera& c = s.camera;
    fprintf(f, "camera"); hv3(f, c.pos); hv3(f, c.forward); hv3(f, c.up);
    hv(f, c.xResolution); hv(f, c.yResolution); hv(f, c.imagePlaneDist); fprintf(f, "\n");
    fprintf(f, "w2r"); for (int i = 0; i < 16; i++) hv(f, c.worldToRaster.m.m[i / 4][i % 4]); fprintf(f, "\n");
    fprintf(f, "r2w"); for (int i = 0; i < 16; i++) hv(f, c.rasterToWorld.m.m[i / 4][i % 4]); fprintf(f, "\n");
    fprintf(f, "sphere"); hv3(f, s.sceneSphere.sceneCenter); hv(f, s.sceneSphere.sceneRadius);
    hv(f, s.sceneSphere.invSceneRadiusSqr); fprintf(f, "\n");
    fprintf(f, "totarea"); hv(f, s.totArea); fprintf(f, "\n");
    if (s.objs.empty()) return;
    fprintf(f, "kd %d", s.kdtreeAccel.depMax);
    hv3(f, s.kdtreeAccel.root->box.l); hv3(f, s.kdtreeAccel.root->box.r); fprintf(f, "\n");
    dump_tree(f, s.kdtreeAccel.root);
}

static void cmd_rays(Scene& s, const char* corpus) {
    FILE* in = fopen(corpus, "rb");
    if (!in) { fprintf(stderr, "no corpus\n"); exit(2); }
    float r[9];
    while (fread(r, sizeof(float), 9, in) == 9) {
        Vector3 o(r[0], r[1], r[2]), d(r[3], r[4], r[5]), tgt(r[6], r[7], r[8]);
        Ray ray(o, d);
        Intersection inter;
        Geometry* g = s.intersect(ray, inter);
        if (g) {
            printf("%d", g_index[g]);
            hv(stdout, inter.t); hv3(stdout, inter.p); hv3(stdout, inter.n);
            printf(" %d %d", inter.inside, inter.matId);
        } else {
            printf("-1");
        }
        printf(" occ %d\n", (int)s.occluded(o, d, tgt));
    }
    fclose(in);
}

static void cmd_kat(Scene& s, int n, unsigned seed) {
    RNG rng(seed);
    FILE* f = stdout;
    // samplers + frame + fresnel
    for (int i = 0; i < n; i++) {
        Vector3 u = rng.randVector3();
        Real pdf = -1.f;
        Vector3 a = sampleCosHemisphere(u, &pdf);
        fprintf(f, "cosh"); hv3(f, u); hv3(f, a); hv(f, pdf); fprintf(f, "\n");
        Real power = 1.f + 200.f * rng.randFloat();
        Vector3 b = samplePowerCosHemisphere(u, power, &pdf);
        Real pp = powerCosHemispherePdf(Vector3(0, 0, 1), b, power);
        fprintf(f, "pcosh"); hv3(f, u); hv(f, power); hv3(f, b); hv(f, pdf); hv(f, pp); fprintf(f, "\n");
        Vector3 p0 = rng.randVector3(), p1 = rng.randVector3(), p2 = rng.randVector3();
        Vector3 t = sampleTriangle(u, p0, p1, p2);
        fprintf(f, "tri"); hv3(f, u); hv3(f, p0); hv3(f, p1); hv3(f, p2); hv3(f, t); fprintf(f, "\n");
        Vector3 z = sampleUniformSphere(rng.randVector3(), NULL);
        Frame fr; fr.buildFromZ(z);
        fprintf(f, "frame"); hv3(f, z); hv3(f, fr.x); hv3(f, fr.y); hv3(f, fr.z); fprintf(f, "\n");
        Real ci = 2.f * rng.randFloat() - 1.f, idx = 1.f + rng.randFloat();
        fprintf(f, "fresnel"); hv(f, ci); hv(f, idx); hv(f, fresnelDielectric(ci, idx)); fprintf(f, "\n");
        int k = (int)(rng.randFloat() * 512), tot = 512;
        Vector3 v0(3.f, 4.f, 0.f), v1(4.f, 4.f, 0.f), v2(3.f, 5.f, 0.f);
        Vector3 st = sampleRectangleStratified(u, v0, v1, v2, k, tot);
        fprintf(f, "strat %d %d", k, tot); hv3(f, u); hv3(f, st); fprintf(f, "\n");
    }
    // BSDF per material
    for (size_t m = 1; m < s.materials.size(); m++) {
        for (int i = 0; i < n; i++) {
            Vector3 nrm = sampleUniformSphere(rng.randVector3(), NULL);
            Vector3 wi = sampleUniformSphere(rng.randVector3(), NULL);
            Vector3 wo = sampleUniformSphere(rng.randVector3(), NULL);
            Vector3 r3 = rng.randVector3();
            Intersection inter;
            inter.n = nrm; inter.matId = (int)m; inter.t = 1.f; inter.inside = 0;
            BSDF b(wi, inter, s);
            fprintf(f, "bsdf %d", (int)m); hv3(f, nrm); hv3(f, wi); hv3(f, wo); hv3(f, r3);
            fprintf(f, " valid %d", (int)b.isValid());
            if (b.isValid()) {
                fprintf(f, " %d", (int)b.isDelta); hv(f, b.cosWi()); hv(f, b.continueProb);
                hv(f, b.fresnelReflect); hv(f, b.componentProb.diffuseProb); hv(f, b.componentProb.glossyProb);
                hv(f, b.componentProb.reflectProb); hv(f, b.componentProb.transProb);
                Real cw = -7.f, dp = -7.f, rp = -7.f;
                Color3 fv = b.f(s, wo, cw, &dp, &rp);
                fprintf(f, " f"); hc3(f, fv); hv(f, cw); hv(f, dp); hv(f, rp);
                fprintf(f, " pdf"); hv(f, b.pdf(s, wo, false)); hv(f, b.pdf(s, wo, true));
                Vector3 ow(-7.f); Real spdf = -7.f, scw = -7.f; int ty = -7;
                Color3 sv = b.sample(s, r3, ow, spdf, scw, &ty);
                fprintf(f, " smp %d", ty); hc3(f, sv); hv3(f, ow); hv(f, spdf); hv(f, scw);
            }
            fprintf(f, "\n");
        }
    }
    // area lights
    Vector3 bl = s.kdtreeAccel.root->box.l, br = s.kdtreeAccel.root->box.r;
    for (size_t li = 0; li < s.lights.size(); li++) {
        AbstractLight* l = s.lights[li];
        for (int i = 0; i < n; i++) {
            Vector3 u = rng.randVector3();
            Vector3 pos = bl + ((br - bl) | u);
            Vector3 r3 = rng.randVector3();
            Vector3 dtl; Real dist = -7.f, dpdf = -7.f, epdf = -7.f, cal = -7.f;
            Color3 il = l->illuminance(s.sceneSphere, pos, r3, dtl, dist, dpdf, &epdf, &cal);
            fprintf(f, "illu %d", (int)li); hv3(f, pos); hv3(f, r3); hc3(f, il); hv3(f, dtl);
            hv(f, dist); hv(f, dpdf); hv(f, epdf); hv(f, cal); fprintf(f, "\n");
            Vector3 dr = rng.randVector3(), pr = rng.randVector3();
            Vector3 ep, ed; Real emp = -7.f, dpa = -7.f, cal2 = -7.f;
            Color3 em = l->emit(s.sceneSphere, dr, pr, ep, ed, emp, &dpa, &cal2);
            fprintf(f, "emit %d", (int)li); hv3(f, dr); hv3(f, pr); hc3(f, em); hv3(f, ep); hv3(f, ed);
            hv(f, emp); hv(f, dpa); hv(f, cal2); fprintf(f, "\n");
            Vector3 rd = sampleUniformSphere(rng.randVector3(), NULL);
            Real gpa = -7.f, gep = -7.f;
            Color3 gr = l->getRadiance(s.sceneSphere, rd, ep, &gpa, &gep);
            fprintf(f, "rad %d", (int)li); hv3(f, rd); hv3(f, ep); hc3(f, gr); hv(f, gpa); hv(f, gep);
            fprintf(f, "\n");
        }
    }
    // camera
    Camera& c = s.camera;
    for (int i = 0; i < n; i++) {
        Vector3 u = rng.randVector3();
        Real x = u.x * c.xResolution, y = u.y * c.yResolution;
        Ray r = c.generateRay(x, y);
        Vector3 w = bl + ((br - bl) | rng.randVector3());
        Vector3 ras = c.worldToRaster.tPoint(w);
        fprintf(f, "cam"); hv(f, x); hv(f, y); hv3(f, r.origin); hv3(f, r.dir); hv3(f, w); hv3(f, ras);
        fprintf(f, " %d\n", (int)c.checkRaster(ras.x, ras.y));
    }
}

static void dump_film(ImageFilm* film, const char* out) {
    FILE* f = fopen(out, "wb");
    for (int i = 0; i < film->height; i++)
        for (int j = 0; j < film->width; j++) {
            float v[3] = {film->color[i][j].r, film->color[i][j].g, film->color[i][j].b};
            fwrite(v, sizeof(float), 3, f);
        }
    fclose(f);
}

static double now() {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// refdrv image: the reference's own ImageFilm / Color3 members on a loaded film
static int cmd_image(int argc, char** argv) {
    if (argc < 8) { fprintf(stderr, "usage: refdrv image H W ITERS TRANSPOSE IN.f32 OUT.rgb\n"); return 2; }
    const int h = atoi(argv[2]), w = atoi(argv[3]), iters = atoi(argv[4]), tr = atoi(argv[5]);
    ImageFilm film(h, w);
    FILE* f = fopen(argv[6], "rb");
    if (!f) { perror(argv[6]); return 1; }
    for (int i = 0; i < h; i++)
        for (int j = 0; j < w; j++) {
            float v[3];
            if (fread(v, sizeof(float), 3, f) != 3) { fprintf(stderr, "short film\n"); return 1; }
            film.color[i][j] = Color3(v[0], v[1], v[2]);
        }
    fclose(f);
    if (tr)  // the in-place swap of bidirPathTracing.cpp:31-41 (square films)
        for (int i = 0; i < h; i++)
            for (int j = 0; j < i; j++) {
                Color3 t = film.color[i][j];
                film.color[i][j] = film.color[j][i];
                film.color[j][i] = t;
            }
    // film->outputImage(filename, 1.f / iterations, 2.2) up to cvSaveImage
    // (film.cpp:45-60); PT passes (1.f, 2.2f), i.e. ITERS = 1
    const Real scale = 1.f / iters, gamma = 2.2;
    film.scale(scale);
    film.clamp();
    film.gamma(gamma);
    FILE* o = fopen(argv[7], "wb");
    if (!o) { perror(argv[7]); return 1; }
    for (int i = 0; i < h; i++)
        for (int j = 0; j < w; j++) {
            unsigned char px[3] = {film.color[i][j].R(), film.color[i][j].G(), film.color[i][j].B()};
            fwrite(px, 1, 3, o);
        }
    fclose(o);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: see header\n"); return 2; }
    const char* cwd = getenv("REFDRV_CWD");
    std::string cmd = argv[1];
    if (cmd == "image") return cmd_image(argc, argv);
    if (cmd == "mt") {
        RNG rng((uint32_t)strtoul(argv[2], 0, 10));
        int n = atoi(argv[3]);
        for (int i = 0; i < n; i++) printf("%u\n", rng.randUInt());
        return 0;
    }
    Parameters para;
    para.load_parameters(argv[3]);
    if (cwd && chdir(cwd) != 0) { perror("chdir"); }
    if (cmd == "scene" || cmd == "rays" || cmd == "kat") {
        Scene* s = new Scene();
        s->init(argv[2], para);
        index_objs(*s);
        if (cmd == "scene") cmd_scene(*s);
        else if (cmd == "rays") cmd_rays(*s, argv[4]);
        else cmd_kat(*s, atoi(argv[4]), (unsigned)strtoul(argv[5], 0, 10));
        return 0;
    }
    if (cmd == "bdpt") {
        BidirPathTracing* b = new BidirPathTracing();
        b->init(argv[2], para);
        b->iterations = atoi(argv[4]);
        b->rng.seed((uint32_t)strtoul(argv[5], 0, 10));
        double t0 = now();
        b->render();
        double t1 = now();
        dump_film(b->film, argv[6]);
        printf("render_seconds %.6f\n", t1 - t0);
        return 0;
    }
    if (cmd == "vcm") return refdrv_vcm(argc, argv, para);
    if (cmd == "pt") {
        PathIntegrator* p = new PathIntegrator();
        p->init(argv[2], para);
        p->rng.seed((uint32_t)strtoul(argv[4], 0, 10));
        double t0 = now();
        p->render();
        double t1 = now();
        dump_film(p->film, argv[5]);
        printf("render_seconds %.6f\n", t1 - t0);
        return 0;
    }
    fprintf(stderr, "unknown command\n");
    return 2;
}
