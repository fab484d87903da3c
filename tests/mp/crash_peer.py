import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ['MPIT_CPU_ONLY'] = '1'
import mpit_amd as mp, torch
mp.Init()
W = mp.COMM_WORLD()
if W.Get_rank() == 1:
    os._exit(9)   # crash without Finalize
t = torch.zeros(1)
W.Recv(t, 1, 5)   # would block forever without failure detection
print("should not get here")
