#!/bin/bash
set -o pipefail
bash scripts/pmc_r2.sh r2b && bash scripts/profile.sh r2c2b && echo all-done
