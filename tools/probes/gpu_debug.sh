cd $GRAFT_REPO_ROOT
echo "== no torch"
timeout 120 python -c "
import sys; sys.path.insert(0,'hpg-fastq_amd'); import hpgfastq as H
print('devices', H.lib.hpgq_device_count())
e=H.Engine(H.stats_params(lmax=150)); print('open ok'); e.close()
"
echo "== torch imported first, no cuda init"
timeout 120 python -c "
import torch, sys; sys.path.insert(0,'hpg-fastq_amd'); import hpgfastq as H
print('devices', H.lib.hpgq_device_count())
e=H.Engine(H.stats_params(lmax=150)); print('open ok'); e.close()
print('torch cuda', torch.cuda.is_available())
x=torch.ones(4,device='cuda'); print(x.sum().item())
"
echo "== torch cuda init first"
timeout 120 python -c "
import torch, sys; print(torch.cuda.is_available()); sys.path.insert(0,'hpg-fastq_amd'); import hpgfastq as H
print('devices', H.lib.hpgq_device_count())
e=H.Engine(H.stats_params(lmax=150)); print('open ok'); e.close()
"
echo "== hpgq first then torch"
timeout 120 python -c "
import sys; sys.path.insert(0,'hpg-fastq_amd'); import hpgfastq as H
import torch
print('devices', H.lib.hpgq_device_count())
e=H.Engine(H.stats_params(lmax=150)); print('open ok'); e.close()
print('torch cuda', torch.cuda.is_available())
"
