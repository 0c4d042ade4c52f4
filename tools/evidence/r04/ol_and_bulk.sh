#!/bin/bash
set -o pipefail
./tools/evidence/r04/shard_bulk.sh && ./tools/evidence/r04/other_lines.sh
