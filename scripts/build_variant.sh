#!/bin/bash
# Build libwinmad_rt.so with extra -D flags into winmad-s-raytracer-v1.0_amd/variants/<name>.so
# (select it at run time with WR_LIB=...).  Usage: scripts/build_variant.sh NAME -DFOO=1 ...
# The flags reach the device code and the host BVH build (wr_bvh.cpp).
set -e
cd "$(dirname "$0")/../winmad-s-raytracer-v1.0_amd"
name=$1; shift
mkdir -p variants
make -s build/wr_scene.o build/wr_image.o build/wr_checkpoint.o
g++ -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I../include -Icsrc "$@" \
  -c csrc/wr_bvh.cpp -o variants/$name.bvh.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I../include -Icsrc \
  --offload-arch=gfx950 "$@" -c csrc/wr_render.hip -o variants/$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o variants/$name.so variants/$name.o variants/$name.bvh.o \
  build/wr_scene.o build/wr_image.o build/wr_checkpoint.o -lpthread -ldl
rm -f variants/$name.o variants/$name.bvh.o
echo "variants/$name.so"
