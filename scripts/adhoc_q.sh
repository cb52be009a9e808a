cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/cw6
timeout -k 10 300 python3 -u scripts/ab.py --cfg C2 --frames 16 --steps 5 vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_cw6.so vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_cw6.so 2>&1 | grep -v amdgpu.ids || exit $?
VRHIP_LIB=$PWD/variants/libvrhip_cw6.so timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cw6/write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-roof --interactive-frames 0 --strong-steps 0 --config C2 > gpurun_out/cw6/write.log 2>&1 || exit $?
echo done
