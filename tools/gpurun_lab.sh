#!/bin/bash
# Run a lab command on the GPU box WITH the lab code objects (tools/lab_build/*.hsaco,
# excluded from ordinary pushes by .gpurunignore): drops that line for this one call
# and restores it afterwards, whatever the call's outcome.  Runs HERE, not on the box:
#   tools/gpurun_lab.sh --timeout 600 -- 'TAG=r05x bash tools/gpu.sh declab'
set -u
cd "$(dirname "$0")/.."
cp .gpurunignore /tmp/gpurunignore.keep
trap 'cp /tmp/gpurunignore.keep .gpurunignore' EXIT
grep -v '^tools/lab_build/\*\.hsaco$' /tmp/gpurunignore.keep > .gpurunignore
/usr/local/graft/bin/gpurun "$@"
