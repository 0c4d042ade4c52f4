#!/bin/bash
set -e
bash tools/r03b.sh r03b
bash tools/r03c.sh r03c
echo all-ok
