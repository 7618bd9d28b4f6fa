"""cProfile of the whole PG-MORL run of bench.py's whole-run leg (GPU box): where the host time goes around the
device iterations (generation setup, record unpack, EP / population / selection, writer, final artefacts).
Usage: python scripts/prof_whole.py [out.txt]"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_whole.txt'
args = argparse.Namespace(whole_run_steps=5e6, tasks=40, num_processes=4, num_steps=2048)
bench.whole_run(args, 40e6)  # warm: library load, allocator, first compilation of nothing (all AOT)
pr = cProfile.Profile()
pr.enable()
res = bench.whole_run(args, 40e6)  # (iter_value only scales the reported ratio)
pr.disable()
s = io.StringIO()
st = pstats.Stats(pr, stream=s)
st.sort_stats('cumulative').print_stats(45)
st.sort_stats('tottime').print_stats(35)
with open(out, 'w') as f:
    f.write(json.dumps({k: v for k, v in res.items() if k != 'generation_rl_host_s'}) + '\n')
    f.write(json.dumps(res['generation_rl_host_s']) + '\n')
    f.write(s.getvalue())
print(json.dumps({k: v for k, v in res.items() if k != 'generation_rl_host_s'}))
