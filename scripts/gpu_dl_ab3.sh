set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_dl_ab.sh dlt_mb "libbugseg.so libbugseg.so@BUGSEG_DL_GTM=0" "--batch 64 --steps 10" &&
bash scripts/gpu_dl_ab.sh dlt_rn "libbugseg.so libbugseg.so@BUGSEG_DL_GTM=0" "--backbone resnet_v1_101_beta --batch 16 --steps 10" &&
bash scripts/gpu_dl_ab.sh dlt_xc "libbugseg.so libbugseg.so@BUGSEG_DL_GTM=0" "--backbone xception_65 --batch 32 --steps 10"
