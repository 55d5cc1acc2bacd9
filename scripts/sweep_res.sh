set -o pipefail
cd $GRAFT_REPO_ROOT
for c in 1 2 4; do echo "NXHIP_RES_CHUNKS=$c"; NXHIP_RES_CHUNKS=$c timeout -k 10 200 python -u scripts/direct_timing.py 15 15 100 2>&1 | grep direct; done
for c in 1 4; do echo "C4 NXHIP_RES_CHUNKS=$c"; NXHIP_RES_CHUNKS=$c timeout -k 10 300 python -u scripts/direct_timing.py 18 19 20 2>&1 | grep direct; done
for j in 128 512; do echo "NXHIP_PC_JOBS=$j"; NXHIP_PC_JOBS=$j timeout -k 10 200 python -u scripts/direct_timing.py 15 15 100 2>&1 | grep direct; done
for j in 512 1024 2048; do echo "C4 NXHIP_PC_JOBS=$j"; NXHIP_PC_JOBS=$j timeout -k 10 300 python -u scripts/direct_timing.py 18 19 20 2>&1 | grep direct; done
