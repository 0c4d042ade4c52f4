#!/bin/bash
set -o pipefail
./tools/evidence/r04/prio_k20.sh && ./tools/evidence/r04/final.sh
