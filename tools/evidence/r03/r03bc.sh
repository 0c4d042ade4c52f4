#!/bin/bash
set -e
bash tools/evidence/r03/r03b.sh r03b
bash tools/evidence/r03/r03c.sh r03c
echo all-ok
