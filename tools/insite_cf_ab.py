"""Diagnostic (GPU): sampled-row status / iteration agreement of the INSITE bench cohort with the oracle for the
library in use (INSITE_LIB_OVERRIDE selects a variant build, e.g. -DINSITE_REFINE_CF=0).  Not product code."""
# A/B: the bench cohort's sampled-row status agreement with the oracle, CF=1 (default lib) vs CF=0 (variant lib)
import os, sys, json
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import bench, torch
from insite_amd import ops
def main():
    dev = torch.device("cuda", 0)
    coh, V, arm, sl, c0, dt = bench.insite_rows(1_000_000, 60, 1, dev)
    plan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5)
    preds, coef, status, iters = plan()
    torch.cuda.synchronize()
    o = plan.order.long()
    par = bench.insite_parity(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, preds, coef, status, iters,
                              extra=(o[:64].cpu().numpy(), o[-64:].cpu().numpy()))
    print(os.environ.get("INSITE_LIB_OVERRIDE", "default"), json.dumps({k: v for k, v in par.items() if k not in ("oracle", "cohort")}))
if __name__ == "__main__":
    main()
