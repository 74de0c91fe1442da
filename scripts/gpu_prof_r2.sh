#!/bin/bash
# round-2 profiles: config-2 headline and config-3 with the node exchange (kernel trace + FETCH/WRITE passes)
set -o pipefail
bash scripts/profile.sh r2c2 && echo c2-done && bash scripts/profile.sh r2c3x --config 3 --exchange && echo c3x-done
