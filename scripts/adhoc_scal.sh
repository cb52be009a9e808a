cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/tile_scaling.py C5 16 0 1,4,8 2>&1 | grep -v amdgpu.ids | sed 's/^/auto /' || exit $?
TS_OVERLAP=1 timeout -k 10 300 python3 -u scripts/tile_scaling.py C5 16 0 1,4,8 2>&1 | grep -v amdgpu.ids | sed 's/^/ovl1 /' || exit $?
timeout -k 10 200 python3 -u scripts/critical_path.py C2,C3 1280x720 2>&1 | grep -v amdgpu.ids
