#!/bin/bash
# Build an A/B variant of the native library with extra compile flags:
#   tools/ab_build.sh <name> "<flags>"  ->  lpcnet_amd/liblpcnet_mi355x_<name>.so
# (load it with LPCNET_LIB_VARIANT=<name>; never the default library)
set -e
cd "$(dirname "$0")/.."
make -s lib BUILD=build_ab_$1 LIB=lpcnet_amd/liblpcnet_mi355x_$1.so EXTRA="$2" -j8
echo "built lpcnet_amd/liblpcnet_mi355x_$1.so with: $2"
