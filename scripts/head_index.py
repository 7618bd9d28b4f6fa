"""Enter PMC / SQ summaries into the HEAD indexes bench.py quotes (profiles/pmc_head.json, profiles/sq_head.json):
one entry per workload, keeping the summary's variant and kernel-source hash (bench quotes an entry only for the
same launch and sources).  Measurement tool, not product code.
    python scripts/head_index.py pmc profiles/r06g_pmc_walker_p40.json ...
    python scripts/head_index.py sq profiles/r06g_sq_walker_p40.json ..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = {'pmc': "The PMC summary (scripts/pmc_summary.py) bench.py quotes as roofline.traffic, one per workload. An entry is "
              "quoted only for the exact launch it measured: 'variant' = the pgm_ppo_update_variant string and "
              "'source_hash' = bench.kernel_source_hash of that kernel's sources; re-take it whenever either changes. "
              "A/B files (other maps or variants) are never listed here.",
       'sq': "The SQ-counter summary (scripts/sq_summary.py) bench.py quotes as roofline.limiter / mfma_busy, one per "
             "workload, under the same variant + source-hash rule as pmc_head.json."}


def main():
    kind, files = sys.argv[1], sys.argv[2:]
    path = os.path.join(ROOT, 'profiles', f'{kind}_head.json')
    idx = json.load(open(path)) if os.path.exists(path) else {'_doc': DOC[kind], 'entries': {}}
    for f in files:
        d = json.load(open(f))
        if not d.get('variant') or not d.get('source_hash'):
            raise SystemExit(f'{f}: no variant / source hash recorded')
        ent = {'variant': d['variant'], 'source_hash': d['source_hash'], 'source': os.path.relpath(f, ROOT)}
        if kind == 'pmc':
            ent['hbm_bytes_per_launch'] = d['hbm_bytes_per_launch']
        else:
            ent.update({k: d.get(k) for k in ('mfma_busy_share', 'wait_any_share', 'lds_bank_conflict_per_active_lds',
                                                'kernel_ns_profiled')})
        idx['entries'][d['workload']] = ent
        print(d['workload'], ent)
    json.dump(idx, open(path, 'w'), indent=1)


if __name__ == '__main__':
    main()
