import os, sys, torch
sys.path.insert(0, os.getcwd())
from detectron2_tensorflow_amd.config import get_cfg, finalize
from detectron2_tensorflow_amd.modeling import build_model
cfg=get_cfg(); cfg.merge_from_file('configs/COCO-Detection/faster_rcnn_R_50_FPN_1x.yaml'); cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT='raw'
finalize(cfg, False, 1, {'num_thing_classes':80,'num_stuff_classes':53,'stuff_ignore_value':0})
torch.manual_seed(0); m=build_model(cfg).cuda().eval()
img=torch.rand(2,320,480,3,device='cuda')*255
inp={'image':img,'image_shape':torch.tensor([[320,480],[300,470]],device='cuda')}
with torch.no_grad():
    res=[]
    for it in range(3):
        ims=m.preprocess_image(inp); bb=m.backbone(ims.tensor); fp=m.neck(bb)
        props,_,_=m.proposal_generator(ims, fp, None)
        rh=m.roi_heads; feats=[fp[f] for f in rh.in_features]
        boxes=props.boxes; N,P=boxes.shape[:2]
        img_i=torch.arange(N,dtype=torch.int32,device='cuda').repeat_interleave(P)
        x=rh.box_pooler.pool(feats, boxes.reshape(-1,4), img_i); h=rh.box_head(x); lg,dl=rh.box_predictor(h)
        res.append(dict(bb={k:v.clone() for k,v in bb.items()}, fp={k:v.clone() for k,v in fp.items()}, pb=props.boxes.clone(), pool=x.clone(), h=h.clone(), lg=lg.clone()))
    for it in (1,2):
        a,b=res[0],res[it]
        print(it, 'bb', [torch.equal(a['bb'][k],b['bb'][k]) for k in a['bb']], 'fpn', [torch.equal(a['fp'][k],b['fp'][k]) for k in a['fp']],
              'props', torch.equal(a['pb'],b['pb']), 'pool', torch.equal(a['pool'],b['pool']), 'head', torch.equal(a['h'],b['h']), 'logits', torch.equal(a['lg'],b['lg']))
