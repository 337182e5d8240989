import torch, time
from t2omca_amd.learner import TDLearner
from t2omca_amd.modules import TransformerAgent, TransformerMixer
from t2omca_amd.synthetic import make_args, make_batch
dev = torch.device("cuda", 0)
torch.manual_seed(0)
margs = make_args(8, device="cuda")
lr = TDLearner(TransformerAgent(None, margs).to(dev), TransformerMixer(margs).to(dev), precision="bf16")
batch, w = make_batch(64, 20, 8, seed=1, device=dev)
t = time.time(); info = lr.train(batch, 0, 0, per_weight=w); torch.cuda.synchronize()
print("pair-barrier smoke ok", float(info["loss_sum"]), time.time() - t, flush=True)
