#!/bin/bash
# Debug probe library (not part of the product): scripts/probes/liblds_guard.so
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 lds_guard.hip -o liblds_guard.so
