#!/bin/bash
# round 4: per-phase lane-cycles of K1 (ACS_PHASE_PROF build) on c3 (1-2 roles) vs c3r1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_r}
mkdir -p $O
timeout -k 10 400 python3 tools/phase_prof.py c3 10000000 0.5 > $O/phase_c3.json 2> $O/phase_c3.err || exit $?
timeout -k 10 400 python3 tools/phase_prof.py c3 10000000 0.0 > $O/phase_c3r1.json 2> $O/phase_c3r1.err || exit $?
cat $O/phase_c3.json $O/phase_c3r1.json
