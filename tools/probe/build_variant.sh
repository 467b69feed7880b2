#!/bin/bash
# Build a variant of the GPU library with extra compile flags on k_encrypt.hip, or on the source
# SRC names (SRC=k_decrypt.hip ...) (probe A/B;
# the other objects come from the product build):
#   bash tools/probe/build_variant.sh <name> <flags...>  ->  fpnn_amd/libfpnn_aes_gpu_<name>.so
# Run the product `make` first.  Load it with FPNN_AES_GPU_LIB (tools/gpu.sh abframes:<lib>).
set -e
cd "$(dirname "$0")/../../fpnn_amd/csrc"
name=$1; shift
mkdir -p build/variant_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" \
  -c ${SRC:-k_encrypt.hip} -o build/variant_$name/${SRC:-k_encrypt.hip}.o
objs=$(ls build/*.hip.o build/*.host.o | grep -v "/${SRC:-k_encrypt.hip}.o\$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic $objs build/variant_$name/${SRC:-k_encrypt.hip}.o \
  -o ../libfpnn_aes_gpu_$name.so
echo "built fpnn_amd/libfpnn_aes_gpu_$name.so"
