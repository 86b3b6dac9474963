#!/bin/bash
# A/B build of the library from an earlier commit's kernel source (diagnostic):
#   tools/abbuild_rev.sh <name> <git rev> [-DMACRO=...]...
# builds cndp_amd/lib/libcndp_gpu_<name>.so from <rev>'s cndp_gpu.hip with this tree's
# headers and host sources; select it at run time with CNDP_GPU_LIB (tools/abpairs.sh).
set -e
cd "$(dirname "$0")/.."
name=$1
rev=$2
shift 2
obj=cndp_amd/build/ab_$name
mkdir -p "$obj"
git show "$rev:cndp_amd/csrc/cndp_gpu.hip" > "$obj/cndp_gpu.hip"
gcc -O3 -fPIC -std=gnu11 -c cndp_amd/csrc/rib.c -o "$obj/rib.o"
gcc -O3 -fPIC -std=gnu11 -c cndp_amd/csrc/fib.c -o "$obj/fib.o"
gcc -O3 -fPIC -std=gnu11 -Iinclude -c cndp_amd/csrc/node.c -o "$obj/node.o"
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -w -Icndp_amd/csrc -Iinclude "$@" \
    -c "$obj/cndp_gpu.hip" -o "$obj/cndp_gpu.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--version-script=cndp_amd/csrc/exports.map \
    -o "cndp_amd/lib/libcndp_gpu_$name.so" "$obj/rib.o" "$obj/fib.o" "$obj/node.o" "$obj/cndp_gpu.o" -lpthread
echo "built cndp_amd/lib/libcndp_gpu_$name.so from $rev"
