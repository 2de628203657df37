#!/bin/bash
# Rebuild ONE translation unit of the in-tree library and relink lib/libinsite_hip.so (the build() recipe, one TU).
#   usage: tools/rebuild_tu.sh insite_hip.hip
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
P="$R/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I "$R/include" -c -o "$P/lib/$1.o" "$P/csrc/$1"
OBJS=""
for t in insite_hip.hip insite_ms.hip insite_gen.hip insite_refine.hip insite_rng.hip; do OBJS="$OBJS $P/lib/$t.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$P/lib/libinsite_hip.so.tmp" $OBJS -lhiprtc
mv "$P/lib/libinsite_hip.so.tmp" "$P/lib/libinsite_hip.so"
