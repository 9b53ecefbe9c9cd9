"""Child script for tests/test_launch.py: prints what the launcher handed this rank.
Rank 0 prints one JSON result line like bench.py's; LAC_TEST_FAIL_RANK=r makes rank r fail."""
import json
import os
import sys

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
info = {"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"]), "world": world,
        "master_addr": os.environ.get("MASTER_ADDR"), "argv": sys.argv[1:]}
print("env " + json.dumps(info), flush=True)
if os.environ.get("LAC_TEST_FAIL_RANK") == str(rank):
    sys.exit(7)
if rank == 0:
    print(json.dumps({"metric": "test", "value": 1.0, "n_gpus": world, "argv": sys.argv[1:]}), flush=True)
