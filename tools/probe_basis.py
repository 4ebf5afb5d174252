"""Predictor basis-kernel sub-phases on the config-4 shard (run with CF_MI355X_LIB = a build with
-DCF_PRED_BASIS_PROBE=1): the share of the basis phase spent building the complement W (Omega
products, Cholesky-QR, the row solve) and in the joint orthogonalisation step."""
import os, runpy, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["probe_c4.py", sys.argv[1] if len(sys.argv) > 1 else "125000"]
import collaborative_filtering_amd.api as api
orig = api.Context.debug_phases
def wrapped(self, enable=True, read=False):
    r = orig(self, enable, read)
    if read:
        b = max(r["basis"], 1)
        print(f"basis sub-phases: complement build {r['wide'] / b * 100:.1f}% | joint step {r['gram'] / b * 100:.1f}%"
              f" of basis cycles; basis {r['basis'] / max(r['setup'] + r['basis'] + r['fast'] + r['dense'], 1) * 100:.1f}% of all", flush=True)
    return r
api.Context.debug_phases = wrapped
runpy.run_path("tools/probe_c4.py", run_name="__main__")
