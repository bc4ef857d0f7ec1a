#!/bin/bash
# end-of-round call: the whole GPU suite, the pgr A/B of the flow kernel's
# sliced copy, then the three profiles (PMC on the final sources) and smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh r04n tests || exit 1
TAG=r04v BPC="1 4" NO_C3=1 NO_TESTS=1 bash tools/diag/flow_ell_ab.sh || exit 1
bash tools/gpu_round.sh r04n prof:c2 prof:netlist prof:c4 smoke || exit 1
