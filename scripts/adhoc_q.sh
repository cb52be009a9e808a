cd $GRAFT_REPO_ROOT
run() {  # run <label> <lib> [env...]
  local lab=$1 lib=$2; shift 2
  for c in C2 C3; do
    env "$@" VRHIP_LIB=$PWD/$lib timeout -k 10 200 python3 -u scripts/tile_scaling.py $c 16 0 1,8 2>&1 | grep "N=8" | sed "s|^|$lab |" || return 1
  done
}
run s3_q4 variants/libvrhip_s3.so || exit 1
run s3_q8 variants/libvrhip_s3.so GPU_MAX_HW_QUEUES=8 || exit 1
run s6_q4 variants/libvrhip_s6.so || exit 1
run s6_q8 variants/libvrhip_s6.so GPU_MAX_HW_QUEUES=8 || exit 1

