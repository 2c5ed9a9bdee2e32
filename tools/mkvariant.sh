#!/bin/bash
# A/B variant tree: a copy of this tree (sources, tests, bench) under ab/<name>,
# its library built with EXTRA="<defines>".  Usage: tools/mkvariant.sh name "-DX=1 ..."
set -e
cd "$(dirname "$0")/.."
name=$1; shift
rm -rf ab/$name && mkdir -p ab/$name
tar --exclude=./.git --exclude=./ab --exclude=./gpurun_out --exclude=./tools/_variants \
    --exclude='*.o' --exclude='*.so' --exclude=./profiles --exclude=./tests -cf - . | tar -C ab/$name -xf -
make -s -C ab/$name -j8 EXTRA="$*" >/dev/null
echo "ab/$name: EXTRA=$*"
