#!/bin/bash
# Profiling-only ablation / tuning builds of libinsite_hip.so (never used by product code paths).
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
P="$R/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"
rm -rf "$P/lib/ablate"; mkdir -p "$P/lib/ablate"
build() { /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC "$@" -I "$R/include" -o "$P/lib/ablate/libinsite_hip_$NAME.so" "$P/csrc/insite_hip.hip" "$P/csrc/insite_ms.hip" "$P/csrc/insite_gen.hip" "$P/csrc/insite_refine.hip" "$P/csrc/insite_rng.hip" -lhiprtc & }
for v in ${VARIANTS:-NOSTORE NOARM RT16 RT64}; do
  case $v in
    NOSTORE) NAME=$v build -DINSITE_ABLATE_NOSTORE ;;
    RK45PI) NAME=$v build -DINSITE_RK45_PER_INTERVAL ;;
    RKW8W6) NAME=$v build -DINSITE_RK45_WIN=8 -DINSITE_RK45_WPE=6 ;;
    RKPMNT) NAME=$v build -DINSITE_RK45_PM_NT=1 ;;
    MSV1) NAME=$v build -DINSITE_MS_V1 ;;
    MS4S0) NAME=$v build -DINSITE_MS4_SCHED=0 ;;
    MS4R10) NAME=$v build -DINSITE_MS4_RING=10 ;;
    MS4NOMFMA) NAME=$v build -DINSITE_MS4_ABL_NOMFMA=1 ;;
    MS4FULL) NAME=$v build -DINSITE_MS4_FULLROW=1 ;;
    MS4ZSYNC) NAME=$v build -DINSITE_MS4Z_SYNC=1 ;;
    MS4ZNOSYNC) NAME=$v build -DINSITE_MS4Z_SYNC=0 ;;
    MS4MASKSEL) NAME=$v build -DINSITE_MS4Z_MASKSEL=1 ;;
    MS4PRIO) NAME=$v build -DINSITE_MS4_PRIO=1 ;;
    MS4NC1) NAME=$v build -DINSITE_MS4_NCHUNK=1 ;;
    MS4NOBUF) NAME=$v build -DINSITE_MS4_BUFLD=0 ;;
    MS4NOPACK) NAME=$v build -DINSITE_MS4Z_PACK=0 ;;
    STLSEP) NAME=$v build -DINSITE_STLSQ_SEPARATE ;;
    STEPDEPTH3) NAME=$v build -DINSITE_TM_DEPTH=3 ;;
    GORD1) NAME=$v build -DINSITE_GRAM_ORDER=1 ;;
    STEPITEM) NAME=$v build -DINSITE_STEP_RANGED=0 ;;
    STEPSPLIT) NAME=$v build -DINSITE_STEP_SERIAL=0 ;;
    DR600) NAME=$v build -DINSITE_DEF_RSTATIC=600 ;;
    DR800) NAME=$v build -DINSITE_DEF_RSTATIC=800 ;;
    DR800C2) NAME=$v build -DINSITE_DEF_RSTATIC=800 -DINSITE_DEF_RCHUNK=2 ;;
    DGPRIO) NAME=$v build -DINSITE_DEF_GPRIO=2 ;;
    DGPRIO800) NAME=$v build -DINSITE_DEF_GPRIO=2 -DINSITE_DEF_RSTATIC=800 ;;
    DYN0) NAME=$v build -DINSITE_STEP_DYN_STATIC=0 ;;
    DYN250) NAME=$v build -DINSITE_STEP_DYN_STATIC=250 ;;
    DYN750) NAME=$v build -DINSITE_STEP_DYN_STATIC=750 ;;
    DYN1000) NAME=$v build -DINSITE_STEP_DYN_STATIC=1000 ;;
    DCH1) NAME=$v build -DINSITE_STEP_DYN_CHUNK=1 ;;
    DCH4) NAME=$v build -DINSITE_STEP_DYN_CHUNK=4 ;;
    GSH450) NAME=$v build -DINSITE_STEP_GSHARE=450 ;;
    GSH550) NAME=$v build -DINSITE_STEP_GSHARE=550 ;;
    GSH600) NAME=$v build -DINSITE_STEP_GSHARE=600 ;;
    GRANGED) NAME=$v build -DINSITE_GRAM_RANGED=1 ;;
    GORD1D3) NAME=$v build -DINSITE_GRAM_ORDER=1 -DINSITE_TM_DEPTH=3 ;;
    GT8D4) NAME=$v build -DINSITE_GT=8 -DINSITE_TM_DEPTH=4 ;;
    GNOCOMP) NAME=$v build -DINSITE_ABLATE_GRAM_NOCOMPUTE ;;
    STAGEWISE) NAME=$v build -DINSITE_ROLLOUT_STAGEWISE ;;
    WPE3) NAME=$v build -DINSITE_GRAM_WPE=3 -DINSITE_STEP_WPE=3 ;;
    SWPE3) NAME=$v build -DINSITE_STEP_WPE=3 ;;
    GNS2) NAME=$v build -DINSITE_GRAM_NS_MIN=2 ;;
    GNOGPH) NAME=$v build -DINSITE_ABLATE_NOGPHASE ;;
    GT8D3) NAME=$v build -DINSITE_GT=8 -DINSITE_TM_DEPTH=3 ;;
    GT8D5) NAME=$v build -DINSITE_GT=8 -DINSITE_TM_DEPTH=5 ;;
    MS4NOEMIT) NAME=$v build -DINSITE_MS4_ABL_NOEMIT=1 ;;
    RKW8W8) NAME=$v build -DINSITE_RK45_WIN=8 -DINSITE_RK45_WPE=8 ;;
    RKW16W5) NAME=$v build -DINSITE_RK45_WIN=16 -DINSITE_RK45_WPE=5 ;;
    RKNOSTAGE) NAME=$v build -DINSITE_RK45_STAGE=0 ;;
    RKR02) NAME=$v build -DINSITE_RK45_CLOSE_BRANCH=1 -DINSITE_RK45_ROOT_BRANCH=1 ;;
    RKROOTBR) NAME=$v build -DINSITE_RK45_ROOT_BRANCH=1 ;;
    RKW12) NAME=$v build -DINSITE_RK45_WIN=12 ;;
    RKW8) NAME=$v build -DINSITE_RK45_WIN=8 ;;
    RKW8W5) NAME=$v build -DINSITE_RK45_WIN=8 -DINSITE_RK45_WPE=5 ;;
    RKW4W5) NAME=$v build -DINSITE_RK45_WIN=4 -DINSITE_RK45_WPE=5 ;;
    SEGKC8) NAME=$v build -DINSITE_SEG_KC=8 -DINSITE_SEG_WPE=3 ;;
    SEGTILE) NAME=$v build -DINSITE_SEG_RANGED=0 ;;
    SEGKC8R) NAME=$v build -DINSITE_SEG_KC=8 ;;
    SEGKC4) NAME=$v build -DINSITE_SEG_KC=4 -DINSITE_SEG_WPE=4 ;;
    SEGKC16) NAME=$v build -DINSITE_SEG_KC=16 -DINSITE_SEG_WPE=2 ;;
    SEGNOPF) NAME=$v build -DINSITE_SEG_PF=0 -DINSITE_SEG_WPE=4 ;;
    SEGKC16NOPF) NAME=$v build -DINSITE_SEG_KC=16 -DINSITE_SEG_PF=0 -DINSITE_SEG_WPE=3 ;;
    MSTAIL0) NAME=$v build -DINSITE_MS_TAIL=0 ;;
    MSTAIL1) NAME=$v build -DINSITE_MS_TAIL=1 ;;
    MSTAIL1WPE1) NAME=$v build -DINSITE_MS_TAIL=1 -DINSITE_MS_WPE=1 ;;
    NOARM) NAME=$v build -DINSITE_ABLATE_NOARM ;;
    TIMING) NAME=$v build -DINSITE_TIMING ;;
    LATE) NAME=$v build -DINSITE_GRAM_LATE_ISSUE ;;
    NOMEM) NAME=$v build -DINSITE_ABLATE_NOARM -DINSITE_ABLATE_NOSTORE ;;
    RT16) NAME=$v build -DINSITE_RT=16 ;;
    RT64) NAME=$v build -DINSITE_RT=64 ;;
    NOGPHASE) NAME=$v build -DINSITE_ABLATE_NOGPHASE ;;
    GT32) NAME=$v build -DINSITE_GT=32 ;;
    NS2) NAME=$v build -DINSITE_GRAM_NS_MIN=2 ;;
    NS4) NAME=$v build -DINSITE_GRAM_NS_MIN=4 ;;
    GT32NS2) NAME=$v build -DINSITE_GT=32 -DINSITE_GRAM_NS_MIN=2 ;;
    TG8) NAME=$v build -DINSITE_TG=8 ;;
    TG32) NAME=$v build -DINSITE_TG=32 ;;
    TG64) NAME=$v build -DINSITE_TG=64 ;;
    NOCOMPUTE) NAME=$v build -DINSITE_ABLATE_NOCOMPUTE ;;
    NT) NAME=$v build -DINSITE_STORE_AUX=2 ;;
    SC1) NAME=$v build -DINSITE_STORE_AUX=1 ;;
    NT3) NAME=$v build -DINSITE_STORE_AUX=3 ;;
    PPL1) NAME=$v build -DINSITE_FORCE_PPL=1 ;;
    PPW3) NAME=$v build -DINSITE_PP_WPE=3 ;;
    PPW4) NAME=$v build -DINSITE_PP_WPE=4 ;;
    PPL2) NAME=$v build -DINSITE_FORCE_PPL=2 ;;
    PPL4) NAME=$v build -DINSITE_FORCE_PPL=4 ;;
    RWPE1) NAME=$v build -DINSITE_REFINE_WPE4=1 ;;
    RWPE2) NAME=$v build -DINSITE_REFINE_WPE4=2 ;;
    RWPE3) NAME=$v build -DINSITE_REFINE_WPE4=3 ;;
    RWPE5) NAME=$v build -DINSITE_REFINE_WPE4=5 ;;
    RWPE6) NAME=$v build -DINSITE_REFINE_WPE4=6 ;;
    RWPE8) NAME=$v build -DINSITE_REFINE_WPE4=8 ;;
    RSU1) NAME=$v build -DINSITE_REFINE_SU4=1 ;;
    PREPROWS) NAME=$v build -DINSITE_PREP_ROWS=1 ;;
    RSU1W5) NAME=$v build -DINSITE_REFINE_SU4=1 -DINSITE_REFINE_WPE4=5 ;;
    KWPE5) NAME=$v build -DINSITE_RK45_WPE=5 ;;
    RW8_2) NAME=$v build -DINSITE_REFINE_WPE8=2 ;;
    RREG8) NAME=$v build -DINSITE_REFINE_REG=8 ;;
    RQUAD) NAME=$v build -DINSITE_REFINE_QUAD=1 ;;
    RQUAD5) NAME=$v build -DINSITE_REFINE_QUAD=1 -DINSITE_REFINE_WPE4=5 ;;
    KWPE6) NAME=$v build -DINSITE_RK45_WPE=6 ;;
    KWPE8) NAME=$v build -DINSITE_RK45_WPE=8 ;;
  esac
done
wait
