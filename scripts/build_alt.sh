#!/bin/bash
# build the library at a git revision (default HEAD) into vina-slam_amd/lib_alt/ (for scripts/ab.sh)
set -e
REV=${1:-HEAD}
WT=/tmp/vg_alt_wt
rm -rf $WT; git -C /root/repo worktree prune
git -C /root/repo worktree add -f --detach $WT $REV >/dev/null
make -C $WT/vina-slam_amd -j8 lib/libvina_gpu.so >/dev/null
mkdir -p /root/repo/vina-slam_amd/lib_alt
cp $WT/vina-slam_amd/lib/libvina_gpu.so /root/repo/vina-slam_amd/lib_alt/
git -C /root/repo worktree remove --force $WT
echo "lib_alt <- $(git -C /root/repo rev-parse --short $REV)"
