import numpy as np
d = np.load('gpurun_out/geom.npz')
pl, rg, nc, rec, tq = d['pl'].astype(np.int64), d['ranges'].reshape(-1,2).astype(np.int64), d['n_contrib'], d['rec'], d['tq']
print("pl max", pl.max(), "mask bits present:", (pl >> 28).max())
W,H=1920,1080; gx=120; gy=68
ntiles=gx*gy
tile_of = np.repeat(np.arange(ntiles), rg[:,1]-rg[:,0])
pos = np.arange(len(pl)) - np.repeat(rg[:,0], rg[:,1]-rg[:,0])
gid = pl & ((1<<28)-1)
x,y,A,B,C = [rec[gid,k].astype(np.float64) for k in (0,1,2,3,4)]
t = tq[gid].astype(np.float64)
# quad test (same as quad_mask): min over quadrant rect of d^T(Q - eI)d <= tq
e = 32*5.9604644775390625e-8*(A+C)
a = A-e; c = C-e; b = B
tx = tile_of % gx; ty = tile_of // gx
masks = np.zeros(len(pl), np.int64)
def rect_qmin(x0,x1,y0,y1):
    inside = (x0<=0)&(x1>=0)&(y0<=0)&(y1>=0)
    best = np.full(x0.shape, np.inf)
    nba=-b/a; nbc=-b/c
    for xe in (x0,x1):
        yy=np.clip(nbc*xe, y0, y1); best=np.minimum(best,(a*xe+2*b*yy)*xe+c*yy*yy)
    for ye in (y0,y1):
        xx=np.clip(nba*ye, x0, x1); best=np.minimum(best,(c*ye+2*b*xx)*ye+a*xx*xx)
    return np.where(inside,0.0,best)
bx = tx*16 - x; by = ty*16 - y
for s in range(4):
    x0 = bx + 8*(s&1); y0 = by + 8*(s>>1)
    q = rect_qmin(x0, x0+7, y0, y0+7)
    masks |= ((~(q > t)) | (t<0)*0).astype(np.int64) << s
masks[t < 0] = 0
# per-quadrant n_eff: max n_contrib over quadrant pixels
ncimg = nc.reshape(H,W)
pad = np.zeros((gy*16, gx*16), np.int64); pad[:H,:W] = ncimg
q4 = pad.reshape(gy,16,gx,16)
wm = np.zeros((ntiles,4),np.int64)
for s in range(4):
    sub = q4[:, 8*(s>>1):8*(s>>1)+8, :, 8*(s&1):8*(s&1)+8]
    wm[:,s] = sub.max(axis=(1,3)).reshape(-1)
vis = np.zeros(len(pl), np.int64)
for s in range(4):
    vis |= ((pos < wm[tile_of, s]).astype(np.int64) << s)
mv = masks & vis
pc = lambda m: sum(((m>>s)&1) for s in range(4))
S1 = pc(mv).sum()
top = ((mv & 3) != 0).astype(int); bot = ((mv & 12) != 0).astype(int)
both_top = ((mv & 3) == 3).sum(); both_bot = ((mv & 12) == 12).sum()
print("entries", len(pl), "visited quadrant-iters S1", S1, "(mask only:", pc(masks).sum(), ")")
print("pair(top/bottom) iters", top.sum()+bot.sum(), "of which both-hit", both_top+both_bot)
left = ((mv & 5) != 0).sum(); right = ((mv & 10) != 0).sum()
print("pair(left/right) iters", left+right, "both", ((mv&5)==5).sum()+((mv&10)==10).sum())
print("mask popcount hist", np.bincount(pc(mv), minlength=5))
