#!/bin/bash
# round 6 final: full GPU suite + smoke + bench (tools/r06/full.sh), then the profile set (tools/r06/profiles.sh)
set -o pipefail
bash tools/r06/full.sh || exit $?
bash tools/r06/profiles.sh prof06b || exit $?
