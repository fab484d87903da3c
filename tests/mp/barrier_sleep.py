"""Rank 1 sleeps T_SLEEP seconds before the Barrier the others already wait in (a BiCNN rank
outside the active set, a fast goot worker at the final Barrier): without MPIT_WAIT_TIMEOUT_S
the job completes; with a shorter deadline the waiting ranks abort with the reason."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ['MPIT_CPU_ONLY'] = '1'
import mpit_amd as mp
mp.Init()
W = mp.COMM_WORLD()
if W.Get_rank() == 1:
    time.sleep(float(os.environ.get("T_SLEEP", "4")))
W.Barrier()
print("barrier passed", flush=True)
mp.Finalize()
