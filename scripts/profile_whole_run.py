"""Diagnostic: cProfile of bench.py's whole-run leg (pgmorl_amd.morl.run, Walker pop 40) -- where the host time
between generations goes.  Usage (GPU box): python scripts/profile_whole_run.py > gpurun_out/whole_run_prof.txt"""
import cProfile
import os
import pstats
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

args = types.SimpleNamespace(whole_run_steps=5e6, tasks=40, num_processes=4, num_steps=2048)
bench.whole_run(args, 47.9e6)  # warm: first-call compiles / caches out of the profile
pr = cProfile.Profile()
pr.enable()
r = bench.whole_run(args, 47.9e6)
pr.disable()
print({k: r[k] for k in ('wall_s', 'mopg_s', 'boundary_host_s', 'init_s', 'final_s', 'generations', 'ep_size')})
st = pstats.Stats(pr)
st.sort_stats('cumulative').print_stats(45)
st.sort_stats('tottime').print_stats(30)
