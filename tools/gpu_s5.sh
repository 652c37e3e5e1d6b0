set -e
bash tools/gpu_round.sh s3 "convabs=3,7,13:,tg_ws=1,tg_big=1,tg_big=1;tg_big_persist=1,tg_big=3;tg_big_persist=1,tg_tile_n=256;tg_stages=2;tg_kdepth=32"
DCP_TUNE=tg_ws=1 bash tools/gpu_round.sh s3ws pmc6=3,7,13
