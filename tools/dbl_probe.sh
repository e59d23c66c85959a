#!/bin/bash
# Cost probe of the step's components (bdf_lane.h BCM3_DBL): C3-only library builds that run one
# component twice (results unchanged), timed against the plain build by tools/variant_timing.py:
#   tools/dbl_probe.sh [k ...]        -> varlib/dev_base.so, varlib/dev_dbl<k>.so (default k = 1..9)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
ks=${*:-1 2 3 4 5 6 7 8 9}
"$ROOT/tools/build_popk_variant.sh" dev_base -DBCM3_DEV_TWO_VEC > /dev/null &
for k in $ks; do
  "$ROOT/tools/build_popk_variant.sh" dev_dbl$k -DBCM3_DEV_TWO_VEC -DBCM3_DBL=$k > /dev/null &
done
wait
ls "$ROOT"/varlib/dev_base.so $(for k in $ks; do echo "$ROOT/varlib/dev_dbl$k.so"; done)
