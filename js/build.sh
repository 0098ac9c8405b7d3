#!/bin/sh
# Build the N-API addon js/build/gk_addon.node against libglpk_mi355x.so
# (built by __graft_entry__.build()).  Needs node's headers (/usr/include/node).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$HERE")
NODE_INC=${NODE_INC:-/usr/include/node}
mkdir -p "$HERE/build"
${CC:-gcc} -O2 -fPIC -shared -Wall -I"$NODE_INC" -DNODE_GYP_MODULE_NAME=gk_addon \
    "$HERE/gk_addon.c" -o "$HERE/build/gk_addon.node" \
    -L"$ROOT/glpk.js_amd" -l:libglpk_mi355x.so -Wl,-rpath,'$ORIGIN/../../glpk.js_amd'
