#!/bin/bash
# debugging aid: run the HM engine on one captured picture up to stages 1..5 then in full,
# each in its own process, stopping at the first failure
for st in 1 2 3 4 5 0; do
  AMD_LOG_LEVEL=1 timeout -k 10 120 python -u -m tests.hm_cases 0 stage "$1" "$2" $st || { echo "FAILED at stage $st"; exit 1; }
done
