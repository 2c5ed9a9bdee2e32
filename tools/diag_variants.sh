#!/bin/bash
# Diagnostic builds of libtpe_hip.so with parts of the table scorer switched
# off (tools/_variants/lib<name>.so; load with HYPEROPT_AMD_LIB=...).  Never
# used by the product path or the tests.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_variants
C=hyperopt_amd/csrc
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
others=""
for f in tpe_fit tpe_parzen tpe_score tpe_history tpe_util; do others="$others $C/$f.o"; done
make -s
# each argument: comma-separated macros, e.g. TPE_DIAG_SKIP_SAMPLE,TPE_DIAG_NO_GATHER
for v in "$@"; do
  defs=$(echo "$v" | sed 's/^/-D/; s/,/ -D/g')
  name=$(echo "$v" | sed 's/TPE_DIAG_//g; s/TPE_//g; s/,/+/g; s/=/_/g')
  /opt/rocm/bin/hipcc $F $defs -c $C/tpe_table.hip -o /tmp/diag_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others /tmp/diag_$name.o -o "tools/_variants/lib_$name.so"
done
