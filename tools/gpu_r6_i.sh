#!/bin/bash
# round-6: does the amdsmi sampler thread cost the convergence run (host-heavy init) time?  Alternating, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for tel in 1 0; do
    echo "== round $r telemetry $tel"
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --telemetry $tel | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['convergence']
print(d['ms_per_step'], {k: round(v['wall_s']*1e3, 2) for k, v in c.items()})" || exit 1
  done
done
