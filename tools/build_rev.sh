#!/usr/bin/env bash
# Build librtamd.so of a past commit into raytracinginoneweekendinrust_amd/_lib/old/
# for same-box A/B timing with tools/ab_time.py. Usage: bash tools/build_rev.sh <rev>
set -eu
cd "$(dirname "$0")/.."
rev=$(git rev-parse --short "$1")
out=raytracinginoneweekendinrust_amd/_lib/old/librtamd_$rev.so
[ -f "$out" ] && { echo "$out"; exit 0; }
tmp=$(mktemp -d /tmp/rtrev.XXXXXX)
git worktree add -f "$tmp" "$rev" -q
make -C "$tmp/raytracinginoneweekendinrust_amd/csrc" -j8 ../_lib/librtamd.so > /dev/null
mkdir -p "$(dirname "$out")"
cp "$tmp/raytracinginoneweekendinrust_amd/_lib/librtamd.so" "$out"
git worktree remove --force "$tmp"
echo "$out"
