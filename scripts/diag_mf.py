import os, sys, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "scripts"))
import diag_phases as dp
from qppvm_amd.problem import QPPVMProblem
from qppvm_amd.synth import qppvm_instances, replicate
p1 = QPPVMProblem(n=30, tau_max=1e6)
inp = replicate(qppvm_instances(p1, 1, seed=1), 4096)
diag = os.path.join(dp.ROOT, "qppvm_amd", "libwbq_diag.so")
print(os.environ.get("WBQ_MFMA_MAX_BATCH"), json.dumps(dp.run(diag, p1, inp, stamps=True)))
