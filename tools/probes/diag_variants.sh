#!/bin/bash
# Diagnostic builds of libtpe_hip.so with parts of a kernel switched off or
# swapped (tools/_variants/lib<name>.so; load with HYPEROPT_AMD_LIB=...).
# Never used by the product path or the tests.
#   tools/probes/diag_variants.sh MACRO[,MACRO...] ...   (each argument = one library)
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/_variants
C=hyperopt_amd/csrc
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
make -s
for v in "$@"; do
  defs=$(echo "$v" | sed 's/^/-D/; s/,/ -D/g')
  name=$(echo "$v" | sed 's/TPE_DIAG_//g; s/TPE_//g; s/,/+/g; s/=/_/g')
  objs=""
  for f in tpe_fit tpe_parzen tpe_score tpe_table tpe_history tpe_sorted tpe_prior tpe_dist tpe_util tpe_ops; do
    /opt/rocm/bin/hipcc $F $defs -c $C/$f.hip -o /tmp/diag_${name}_$f.o
    objs="$objs /tmp/diag_${name}_$f.o"
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o "tools/_variants/lib_$name.so"
done
