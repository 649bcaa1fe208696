#!/bin/bash
# variants/NAME/libmml_hip.so: the library with extra compile flags (A/B experiments; load it
# with MML_LIB_PATH=...).  Usage: scripts/build_variant.sh NAME "-DFLAG ..."
# Every variant is an experiments build (-DMML_EXPERIMENTS): its MML_* environment switches
# (MML_HOGWILD_XCD, MML_WRMF_DEBUG, ...) are live; the release library ignores them.
set -e
name=$1; flags="-DMML_EXPERIMENTS ${2:-}"
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/variants/$name  # not under build/: that is gpurun-ignored
mkdir -p "$out"
cd "$root/mymedialite_amd/csrc"
objs=()
for f in *.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include $flags -c -o "$out/${f%.hip}.o" "$f" &
  objs+=("$out/${f%.hip}.o")
done
for f in *.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include $flags -c -o "$out/${f%.cpp}.o" "$f" &
  objs+=("$out/${f%.cpp}.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libmml_hip.so" "${objs[@]}" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f "${objs[@]}"
echo "$out/libmml_hip.so"
