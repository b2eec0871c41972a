#!/bin/bash
# Round 6 final evidence, call A: the GPU suite, smoke, the default line and
# the Large line's timed trace (tools/r06_final.sh part 1), then the FETCH /
# WRITE passes of the zero-copy and materialising decode legs
# (tools/r06_pmc.sh part 1 minus the Large and Small lines, whose dominant
# copies are unchanged since bd8fff8). usage: HONU_COMMIT=<sha> tools/r06_call23.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/r06_final.sh gpurun_out/r06_final 1 || exit $?
bash tools/r06_pmc.sh gpurun_out/r06_pmcfin 3 || exit $?
