"""Worker of the elastic launch test: joins the generation's gloo world, all-reduces a one, records
(world, sum, restart count) and idles until the test drops a 'stop' file."""
import datetime
import os
import sys
import time

import torch
import torch.distributed as dist

out = sys.argv[1]
rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
gen = os.environ['PADDLE_ELASTIC_GEN']
dist.init_process_group('gloo', init_method=f"tcp://{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}",
                        rank=rank, world_size=world, timeout=datetime.timedelta(seconds=30))
t = torch.ones(1)
dist.all_reduce(t)
with open(os.path.join(out, f"gen{gen}_rank{rank}"), 'w') as f:
    f.write(f"{world} {int(t.item())} {os.environ['PADDLE_ELASTIC_RESTART_COUNT']}")
while not os.path.exists(os.path.join(out, 'stop')):
    time.sleep(0.1)
sys.exit(0)
