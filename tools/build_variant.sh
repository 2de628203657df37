#!/bin/bash
# Profiling-only variant builds: recompile ONE translation unit with extra -D flags and link it with the in-tree
# objects of the others -> lib/ablate/libinsite_hip_<NAME>.so (select with INSITE_LIB_OVERRIDE).  Never used by
# product code paths.   usage: tools/build_variant.sh NAME TU.hip [-DFLAG=V ...]
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
P="$R/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"
NAME=$1; TU=$2; shift 2
mkdir -p "$P/lib/ablate"
O="$P/lib/ablate/$NAME.$TU.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -I "$R/include" -c -o "$O" "$P/csrc/$TU"
OBJS=""
for t in insite_hip.hip insite_ms.hip insite_gen.hip insite_refine.hip insite_rng.hip; do
  if [ "$t" = "$TU" ]; then OBJS="$OBJS $O"; else OBJS="$OBJS $P/lib/$t.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$P/lib/ablate/libinsite_hip_$NAME.so" $OBJS -lhiprtc
