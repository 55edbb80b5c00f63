import sys, numpy as np, torch
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/ska-sdp-func_amd'); sys.path.insert(0,'/root/repo/tests')
from oracle import es_oracle
from ska_sdp_func.grid_data import GridderUvwEsFft
dev=torch.device('cuda:0')
n=256; px=2*np.pi/180/n
freq=np.array([1e9],np.float32)
def run(uv):
    R=len(uv)
    uvw=np.zeros((R,3),np.float32); uvw[:,:2]=uv
    vis=(np.arange(R)+1).astype(np.complex64)[:,None]*(1+0.5j)
    wt=np.ones((R,1),np.float32)
    g=[torch.from_numpy(a).to(dev) for a in (uvw,freq,vis,wt)]
    d=torch.zeros((n,n),dtype=torch.float32,device=dev)
    plan=GridderUvwEsFft(*g,d,px,px,1e-5,False)
    G=plan.grid_size
    grid=torch.full((G,G),7.0,dtype=torch.complex64,device=dev)
    plan.grid_scatter(*g,grid)
    geo=es_oracle.geometry_for(uvw,freq,vis,np.zeros((n,n),np.float32),px,1e-5,False)
    ref=es_oracle.scatter(geo,uvw,freq,vis,wt)
    out=grid.cpu().numpy()
    bad=np.argwhere(np.abs(out-ref)>1e-5*np.abs(ref).max())
    print(R, 'G',G,'bad',len(bad))
    for b in bad[:12]:
        print('  cell',b-G//2,'out',out[tuple(b)],'ref',ref[tuple(b)])
scale=299792458.0/(1e9*px*512)   # one grid cell in metres (G=512?)
print('cell m', scale)
run(np.array([[10.3*scale, 20.6*scale]]))
run(np.array([[10.3*scale, 20.6*scale],[12.7*scale, 25.2*scale]]))
run(np.array([[10.3*scale, 20.6*scale],[12.7*scale, 25.2*scale],[-30.1*scale,5.5*scale],[11.1*scale,22.9*scale],[13.4*scale,19.2*scale]]))
