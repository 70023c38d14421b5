#!/bin/bash
# Configure + build everything (daemon, CLI, GPU agent, tests) in ./build.
set -euo pipefail
cd "$(dirname "$0")/.."
cmake -S . -B build -G Ninja -DCMAKE_BUILD_TYPE="${BUILD_TYPE:-RelWithDebInfo}" "$@"
cmake --build build -j "${JOBS:-8}"
