#!/bin/bash
# VAE step: conv / VAE GPU tests, then the A/B of scripts/vae_ab.py (TAG names the output directory)
O=gpurun_out/${TAG:-vae_ab}; cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_vae_train.py tests/test_gpu_vae.py tests/test_abi.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
# shellcheck disable=SC2086
timeout -k 10 400 python -u scripts/vae_ab.py --steps 300 --rounds 3 ${VARIANTS:---variant new: --variant old:ocm.conv.QSUM_FUSED=False,ocm.vae_train.PERSISTENT_ONE=False} > $O/ab.jsonl 2>&1; rc=$?
cat $O/ab.jsonl; exit $rc
