#!/bin/bash
# div_known against IEEE division for EVERY binary32 numerator of the theorem's domain and every
# divisor the step kernel replaces (tests/native/markstein_check.c exhaustive32; ~2.5 min on 8
# host threads): the record tests/test_markstein.py reads, profiles/r05_markstein_exhaustive32.txt.
cd "$(dirname "$0")/.."
gcc -O2 -fopenmp -ffp-contract=off tests/native/markstein_check.c -o /tmp/markstein_check -lm || exit 1
DIVS=$(python3 -c "import sys; sys.path.insert(0, 'tests'); import test_markstein as t; print(' '.join(repr(float(b)) for b in t.divisors()))")
{ echo "# markstein_check exhaustive32 $DIVS"; echo "# (mismatches, numerators tried)"; /tmp/markstein_check exhaustive32 $DIVS; } \
  > profiles/r05_markstein_exhaustive32.txt
cat profiles/r05_markstein_exhaustive32.txt
