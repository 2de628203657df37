set -o pipefail
cd $GRAFT_REPO_ROOT
echo default-joint; DIAG_N=2000 DIAG_JOINT=1 timeout -k 10 120 python tools/coop_diag.py || exit 1
echo nocontract-dense; INSITE_LIB_OVERRIDE=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_NOCONTRACT.so timeout -k 10 120 python tools/coop_diag.py || exit 1
echo nocontract-joint; INSITE_LIB_OVERRIDE=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_NOCONTRACT.so DIAG_N=2000 DIAG_JOINT=1 timeout -k 10 120 python tools/coop_diag.py || exit 1
