import sys, time; sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/oracle')
import soarm_pkg, numpy as np, torch
from lerobot_mujoco_sim2real_amd import mjcf, sim
from oracle import Oracle
for dc in [True, False]:
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML, disable_contact=dc)
    n = 256
    S = sim.BatchSim(cm, n)
    orc = Oracle(cm)
    rng = np.random.default_rng(0)
    iq = rng.uniform(-0.3,0.3,(n,5))
    o_g = S.reset(init_qpos=iq).cpu().numpy()
    st = orc.new_state(n); o_c = orc.reset(st, init_qpos=iq)
    print('dc',dc,'reset obs err', np.abs(o_g-o_c).max())
    for k in range(20):
        a = rng.uniform(-0.5,0.5,(n,5))
        o_g = S.step(a).cpu().numpy(); o_c = orc.step(st, a)
        if k in (0,1,4,19): print(' step',k,'obs err max', np.abs(o_g-o_c).max(), 'median', np.median(np.abs(o_g-o_c)))
    print(' qvel err', np.abs(S.qvel.cpu().numpy().T - st['qvel']).max(), 'status', S.status.cpu().numpy().max(), 'ncon', S.ncon.sum().item(), st['ncon'].sum())
    torch.cuda.synchronize()
    for nn in [4096]:
        S2 = sim.BatchSim(cm, nn); S2.reset()
        a = torch.rand((nn,5), device='cuda')-0.5
        for i in range(3): S2.step(a)
        torch.cuda.synchronize(); t=time.time()
        for i in range(50): S2.step(a)
        torch.cuda.synchronize(); dt=(time.time()-t)/50
        print(' n',nn,'ms/step',dt*1e3,'env-steps/s',nn/dt)
