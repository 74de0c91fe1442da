#!/bin/bash
# Round-2 profiles of the general path (request mix) and of CommandsForKey.update with deps.
set -o pipefail
bash scripts/profile.sh r2mix --accept-frac 0.3 --unordered-frac 0.1 || exit $?
bash scripts/profile.sh r2deps --cfk-update 1000000 --cfk-deps 4 || exit $?
echo profiles-done
