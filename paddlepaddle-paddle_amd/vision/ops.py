"""paddle.vision.ops (reference: python/paddle/vision/ops.py — yolo_loss:58, yolo_box:266,
prior_box:427, box_coder:573, deform_conv2d:753, DeformConv2D:960, distribute_fpn_proposals:1156,
read_file:1301, decode_jpeg:1344, psroi_pool:1393, roi_pool:1514, roi_align:1640, nms:1867,
generate_proposals:2038, matrix_nms:2236).

Detection ops are written as batched tensor programs on the device: RoI ops sample every bin of
every box at once (bilinear gathers), deformable conv is offset-sampled im2col + one GEMM per
group, NMS builds the IoU matrix once and walks it greedily.
"""
import math

import numpy as np
import torch
import torch.nn.functional as TF

from ..core.tensor import Tensor, _wrap, _unwrap
from ..nn.layer.layers import Layer
from ..nn import initializer as I


def _u(x):
    return _unwrap(x) if isinstance(x, Tensor) else x


# ----------------------------------------------------------------- boxes
def _iou_matrix(a, b):
    area_a = (a[:, 2] - a[:, 0]).clamp(min=0) * (a[:, 3] - a[:, 1]).clamp(min=0)
    area_b = (b[:, 2] - b[:, 0]).clamp(min=0) * (b[:, 3] - b[:, 1]).clamp(min=0)
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area_a[:, None] + area_b[None, :] - inter).clamp(min=1e-10)


def _greedy_nms(boxes, scores, thr):
    order = torch.argsort(scores, descending=True)
    b = boxes[order]
    iou = _iou_matrix(b, b)
    n = b.shape[0]
    keep = torch.ones(n, dtype=torch.bool, device=b.device)
    sup = (iou > thr).cpu().numpy()
    k = np.ones(n, dtype=bool)
    for i in range(n):
        if k[i]:
            k[i + 1:] &= ~sup[i, i + 1:]
    keep = torch.from_numpy(k).to(b.device)
    return order[keep]


def nms(boxes, iou_threshold=0.3, scores=None, category_idxs=None, categories=None, top_k=None):
    bx = _u(boxes).float()
    if scores is None:
        sc = torch.arange(bx.shape[0], 0, -1, device=bx.device, dtype=torch.float32)
    else:
        sc = _u(scores).float()
    if category_idxs is None:
        keep = _greedy_nms(bx, sc, iou_threshold)
    else:
        ci = _u(category_idxs)
        cats = (list(categories) if isinstance(categories, (list, tuple)) else _u(categories).tolist()) \
            if categories is not None else ci.unique().tolist()
        parts = []
        for c in cats:
            idx = torch.nonzero(ci == c).squeeze(1)
            if idx.numel():
                parts.append(idx[_greedy_nms(bx[idx], sc[idx], iou_threshold)])
        keep = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.long, device=bx.device)
        keep = keep[torch.argsort(sc[keep], descending=True)]
    if top_k is not None:
        keep = keep[:top_k]
    return _wrap(keep)


def box_coder(prior_box, prior_box_var, target_box, code_type="encode_center_size", box_normalized=True, axis=0,
              name=None):
    pb, tb = _u(prior_box).float(), _u(target_box).float()
    norm = 0.0 if box_normalized else 1.0
    pw = pb[:, 2] - pb[:, 0] + norm
    ph = pb[:, 3] - pb[:, 1] + norm
    px = pb[:, 0] + 0.5 * pw
    py = pb[:, 1] + 0.5 * ph
    if isinstance(prior_box_var, (list, tuple)):
        var = torch.tensor(prior_box_var, device=pb.device, dtype=pb.dtype).expand(pb.shape[0], 4)
    elif prior_box_var is None:
        var = torch.ones_like(pb)
    else:
        var = _u(prior_box_var).float()
    if code_type == "encode_center_size":
        tw = tb[:, 2] - tb[:, 0] + norm
        th = tb[:, 3] - tb[:, 1] + norm
        tx = tb[:, 0] + 0.5 * tw
        ty = tb[:, 1] + 0.5 * th
        out = torch.stack([(tx[:, None] - px[None]) / pw[None] / var[None, :, 0],
                           (ty[:, None] - py[None]) / ph[None] / var[None, :, 1],
                           torch.log((tw[:, None] / pw[None]).abs()) / var[None, :, 2],
                           torch.log((th[:, None] / ph[None]).abs()) / var[None, :, 3]], -1)
        return _wrap(out)
    # decode: target [N, M, 4]; priors broadcast along `axis`
    if tb.dim() == 2:
        tb = tb.unsqueeze(1)
    sh = (1, -1) if axis == 0 else (-1, 1)
    pw_, ph_, px_, py_ = pw.view(sh), ph.view(sh), px.view(sh), py.view(sh)
    v = var.view(sh + (4,)) if var.dim() == 2 else var
    cx = v[..., 0] * tb[..., 0] * pw_ + px_
    cy = v[..., 1] * tb[..., 1] * ph_ + py_
    w = torch.exp(v[..., 2] * tb[..., 2]) * pw_
    h = torch.exp(v[..., 3] * tb[..., 3]) * ph_
    out = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - norm, cy + h / 2 - norm], -1)
    return _wrap(out)


def prior_box(input, image, min_sizes, max_sizes=None, aspect_ratios=[1.0], variance=[0.1, 0.1, 0.2, 0.2],  # noqa: A002,B006
              flip=False, clip=False, steps=[0.0, 0.0], offset=0.5, min_max_aspect_ratios_order=False, name=None):  # noqa: B006
    x, img = _u(input), _u(image)
    fh, fw = x.shape[2], x.shape[3]
    ih, iw = img.shape[2], img.shape[3]
    sw = steps[0] if steps[0] > 0 else iw / fw
    sh = steps[1] if steps[1] > 0 else ih / fh
    ars = [1.0]
    for a in aspect_ratios:
        if all(abs(a - e) > 1e-6 for e in ars):
            ars.append(a)
            if flip:
                ars.append(1.0 / a)
    whs = []
    for i, ms in enumerate(min_sizes):
        if min_max_aspect_ratios_order:
            whs.append((ms, ms))
            if max_sizes:
                m = math.sqrt(ms * max_sizes[i])
                whs.append((m, m))
            for a in ars:
                if abs(a - 1.0) > 1e-6:
                    whs.append((ms * math.sqrt(a), ms / math.sqrt(a)))
        else:
            for a in ars:
                whs.append((ms * math.sqrt(a), ms / math.sqrt(a)))
            if max_sizes:
                m = math.sqrt(ms * max_sizes[i])
                whs.append((m, m))
    dev = x.device
    cy = (torch.arange(fh, device=dev, dtype=torch.float32) + offset) * sh
    cx = (torch.arange(fw, device=dev, dtype=torch.float32) + offset) * sw
    cyy, cxx = torch.meshgrid(cy, cx, indexing='ij')
    wh = torch.tensor(whs, device=dev, dtype=torch.float32)
    boxes = torch.stack([(cxx[..., None] - wh[:, 0] / 2) / iw, (cyy[..., None] - wh[:, 1] / 2) / ih,
                         (cxx[..., None] + wh[:, 0] / 2) / iw, (cyy[..., None] + wh[:, 1] / 2) / ih], -1)
    if clip:
        boxes = boxes.clamp(0, 1)
    var = torch.tensor(variance, device=dev, dtype=torch.float32).expand_as(boxes).contiguous()
    return _wrap(boxes), _wrap(var)


def yolo_box(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox=True, name=None,
             scale_x_y=1.0, iou_aware=False, iou_aware_factor=0.5):
    t, isz = _u(x).float(), _u(img_size)
    N, C, H, W = t.shape
    A = len(anchors) // 2
    if iou_aware:
        ioup = torch.sigmoid(t[:, :A])
        t = t[:, A:]
    t = t.view(N, A, 5 + class_num, H, W)
    an = torch.tensor(anchors, dtype=torch.float32, device=t.device).view(A, 2)
    gy, gx = torch.meshgrid(torch.arange(H, device=t.device), torch.arange(W, device=t.device), indexing='ij')
    bias = -0.5 * (scale_x_y - 1.0)
    cx = (gx + torch.sigmoid(t[:, :, 0]) * scale_x_y + bias) / W
    cy = (gy + torch.sigmoid(t[:, :, 1]) * scale_x_y + bias) / H
    inw, inh = downsample_ratio * W, downsample_ratio * H
    bw = torch.exp(t[:, :, 2]) * an[:, 0].view(1, A, 1, 1) / inw
    bh = torch.exp(t[:, :, 3]) * an[:, 1].view(1, A, 1, 1) / inh
    conf = torch.sigmoid(t[:, :, 4])
    if iou_aware:
        conf = conf ** (1 - iou_aware_factor) * ioup ** iou_aware_factor
    imh, imw = isz[:, 0].float().view(N, 1, 1, 1), isz[:, 1].float().view(N, 1, 1, 1)
    x0, y0 = (cx - bw / 2) * imw, (cy - bh / 2) * imh
    x1, y1 = (cx + bw / 2) * imw, (cy + bh / 2) * imh
    if clip_bbox:
        x0, y0 = x0.clamp(min=0), y0.clamp(min=0)
        x1, y1 = torch.minimum(x1, imw - 1), torch.minimum(y1, imh - 1)
    keep = (conf >= conf_thresh).float()
    boxes = torch.stack([x0, y0, x1, y1], -1) * keep[..., None]
    scores = torch.sigmoid(t[:, :, 5:]) * (conf * keep).unsqueeze(2)
    boxes = boxes.reshape(N, -1, 4)
    scores = scores.permute(0, 1, 3, 4, 2).reshape(N, -1, class_num)
    return _wrap(boxes), _wrap(scores)


def yolo_loss(x, gt_box, gt_label, anchors, anchor_mask, class_num, ignore_thresh, downsample_ratio, gt_score=None,
              use_label_smooth=True, name=None, scale_x_y=1.0):
    """YOLOv3 loss per image: sigmoid-BCE on x/y, L1 on w/h (2 - w*h weighted), objectness with
    ignore-thresh, class BCE (optionally label-smoothed)."""
    t = _u(x).float()
    gb, gl = _u(gt_box).float(), _u(gt_label).long()
    N, C, H, W = t.shape
    mask = list(anchor_mask)
    A = len(mask)
    t = t.view(N, A, 5 + class_num, H, W)
    all_an = torch.tensor(anchors, dtype=torch.float32, device=t.device).view(-1, 2)
    an = all_an[mask]
    inw, inh = downsample_ratio * W, downsample_ratio * H
    gs = _u(gt_score).float() if gt_score is not None else torch.ones(gb.shape[:2], device=t.device)
    bce = TF.binary_cross_entropy_with_logits
    # predicted boxes for the ignore mask
    gy, gx = torch.meshgrid(torch.arange(H, device=t.device), torch.arange(W, device=t.device), indexing='ij')
    px = (gx + torch.sigmoid(t[:, :, 0])) / W
    py = (gy + torch.sigmoid(t[:, :, 1])) / H
    pw = torch.exp(t[:, :, 2]) * an[:, 0].view(1, A, 1, 1) / inw
    ph = torch.exp(t[:, :, 3]) * an[:, 1].view(1, A, 1, 1) / inh
    pred = torch.stack([px - pw / 2, py - ph / 2, px + pw / 2, py + ph / 2], -1).view(N, -1, 4)
    loss = torch.zeros(N, device=t.device)
    obj_target = torch.zeros(N, A, H, W, device=t.device)
    obj_weight = torch.ones(N, A, H, W, device=t.device)
    for n in range(N):
        valid = (gb[n, :, 2] > 0) & (gb[n, :, 3] > 0)
        g = gb[n][valid]
        if g.numel():
            gxyxy = torch.stack([g[:, 0] - g[:, 2] / 2, g[:, 1] - g[:, 3] / 2, g[:, 0] + g[:, 2] / 2,
                                 g[:, 1] + g[:, 3] / 2], -1)
            best_iou = _iou_matrix(pred[n], gxyxy).max(1).values.view(A, H, W)
            obj_weight[n][best_iou > ignore_thresh] = 0
        for j in torch.nonzero(valid).squeeze(1).tolist():
            bx, by, bw, bh = gb[n, j].tolist()
            # best anchor over all anchors by shape IoU
            inter = torch.minimum(all_an[:, 0], torch.tensor(bw * inw)) * torch.minimum(all_an[:, 1],
                                                                                          torch.tensor(bh * inh))
            ious = inter / (all_an[:, 0] * all_an[:, 1] + bw * inw * bh * inh - inter)
            best = int(ious.argmax())
            if best not in mask:
                continue
            a = mask.index(best)
            gi, gj = min(int(bx * W), W - 1), min(int(by * H), H - 1)
            sc = gs[n, j]
            wscale = 2.0 - bw * bh
            tx, ty = bx * W - gi, by * H - gj
            tw = math.log(bw * inw / all_an[best, 0])
            th = math.log(bh * inh / all_an[best, 1])
            cell = t[n, a, :, gj, gi]
            loss[n] = loss[n] + sc * wscale * (bce(cell[0], torch.tensor(tx, device=t.device)) +
                                               bce(cell[1], torch.tensor(ty, device=t.device)) +
                                               (cell[2] - tw).abs() + (cell[3] - th).abs())
            tgt = torch.zeros(class_num, device=t.device)
            pos, neg = (1.0 - 1.0 / class_num, 1.0 / class_num) if use_label_smooth else (1.0, 0.0)
            tgt.fill_(neg)
            tgt[int(gl[n, j])] = pos
            loss[n] = loss[n] + sc * bce(cell[5:], tgt, reduction='sum')
            obj_target[n, a, gj, gi] = sc
            obj_weight[n, a, gj, gi] = 1.0
    obj = bce(t[:, :, 4], obj_target, reduction='none') * obj_weight
    loss = loss + obj.view(N, -1).sum(1)
    return _wrap(loss)


# ----------------------------------------------------------------- RoI ops
def _roi_batch_index(boxes_num, nboxes, device):
    bn = _u(boxes_num)
    if bn is None:
        return torch.zeros(nboxes, dtype=torch.long, device=device)
    return torch.repeat_interleave(torch.arange(bn.numel(), device=device), bn.to(device).long())


def _bilinear(feat, y, x):
    """feat [C, H, W]; y, x same-shaped float grids → [C, *grid]; zero outside (-1, H)."""
    C, H, W = feat.shape
    valid = (y > -1.0) & (y < H) & (x > -1.0) & (x < W)
    y = y.clamp(min=0)
    x = x.clamp(min=0)
    y0 = y.floor().long().clamp(max=H - 1)
    x0 = x.floor().long().clamp(max=W - 1)
    y1 = (y0 + 1).clamp(max=H - 1)
    x1 = (x0 + 1).clamp(max=W - 1)
    y = torch.where(y0 >= H - 1, y0.float(), y)
    x = torch.where(x0 >= W - 1, x0.float(), x)
    ly, lx = y - y0, x - x0
    hy, hx = 1 - ly, 1 - lx
    f = feat.reshape(C, -1)

    def g(yy, xx):
        return f[:, (yy * W + xx).reshape(-1)].reshape((C,) + yy.shape)
    out = g(y0, x0) * (hy * hx) + g(y0, x1) * (hy * lx) + g(y1, x0) * (ly * hx) + g(y1, x1) * (ly * lx)
    return out * valid


def roi_align(x, boxes, boxes_num, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=True, name=None):
    feat, bx = _u(x), _u(boxes).float()
    ph, pw = (output_size, output_size) if isinstance(output_size, int) else output_size
    bidx = _roi_batch_index(boxes_num, bx.shape[0], bx.device)
    off = 0.5 if aligned else 0.0
    outs = []
    for r in range(bx.shape[0]):
        x0, y0, x1, y1 = (bx[r] * spatial_scale - off).tolist()
        rw, rh = x1 - x0, y1 - y0
        if not aligned:
            rw, rh = max(rw, 1.0), max(rh, 1.0)
        bw, bh = rw / pw, rh / ph
        sy = sampling_ratio if sampling_ratio > 0 else int(math.ceil(rh / ph))
        sx = sampling_ratio if sampling_ratio > 0 else int(math.ceil(rw / pw))
        sy, sx = max(sy, 1), max(sx, 1)
        iy = (torch.arange(ph, device=bx.device).view(ph, 1) * bh + y0 +
              (torch.arange(sy, device=bx.device).view(1, sy) + 0.5) * bh / sy).view(ph, sy, 1, 1)
        ix = (torch.arange(pw, device=bx.device).view(pw, 1) * bw + x0 +
              (torch.arange(sx, device=bx.device).view(1, sx) + 0.5) * bw / sx).view(1, 1, pw, sx)
        yy, xx = torch.broadcast_tensors(iy, ix)
        v = _bilinear(feat[bidx[r]].float(), yy, xx)      # [C, ph, sy, pw, sx]
        outs.append(v.mean((2, 4)))
    out = torch.stack(outs) if outs else feat.new_zeros(0, feat.shape[1], ph, pw)
    return _wrap(out.to(feat.dtype))


def roi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    feat, bx = _u(x), _u(boxes).float()
    ph, pw = (output_size, output_size) if isinstance(output_size, int) else output_size
    bidx = _roi_batch_index(boxes_num, bx.shape[0], bx.device)
    H, W = feat.shape[2:]
    outs = []
    for r in range(bx.shape[0]):
        x0, y0, x1, y1 = [int(round(v)) for v in (bx[r] * spatial_scale).tolist()]
        rh, rw = max(y1 - y0 + 1, 1), max(x1 - x0 + 1, 1)
        o = feat.new_zeros(feat.shape[1], ph, pw)
        for i in range(ph):
            hs = min(max(y0 + int(math.floor(i * rh / ph)), 0), H)
            he = min(max(y0 + int(math.ceil((i + 1) * rh / ph)), 0), H)
            for j in range(pw):
                ws = min(max(x0 + int(math.floor(j * rw / pw)), 0), W)
                we = min(max(x0 + int(math.ceil((j + 1) * rw / pw)), 0), W)
                if he > hs and we > ws:
                    o[:, i, j] = feat[bidx[r], :, hs:he, ws:we].amax((1, 2))
        outs.append(o)
    return _wrap(torch.stack(outs) if outs else feat.new_zeros(0, feat.shape[1], ph, pw))


def psroi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    feat, bx = _u(x), _u(boxes).float()
    ph, pw = (output_size, output_size) if isinstance(output_size, int) else output_size
    C = feat.shape[1] // (ph * pw)
    bidx = _roi_batch_index(boxes_num, bx.shape[0], bx.device)
    H, W = feat.shape[2:]
    outs = []
    for r in range(bx.shape[0]):
        x0, y0, x1, y1 = (bx[r] * spatial_scale).tolist()
        x0, y0, x1, y1 = round(x0), round(y0), round(x1) + 1, round(y1) + 1
        rh, rw = max(y1 - y0, 0.1), max(x1 - x0, 0.1)
        o = feat.new_zeros(C, ph, pw)
        for i in range(ph):
            hs = min(max(int(math.floor(y0 + i * rh / ph)), 0), H)
            he = min(max(int(math.ceil(y0 + (i + 1) * rh / ph)), 0), H)
            for j in range(pw):
                ws = min(max(int(math.floor(x0 + j * rw / pw)), 0), W)
                we = min(max(int(math.ceil(x0 + (j + 1) * rw / pw)), 0), W)
                if he > hs and we > ws:
                    ch = torch.arange(C, device=feat.device) * ph * pw + i * pw + j
                    o[:, i, j] = feat[bidx[r], ch, hs:he, ws:we].mean((1, 2))
        outs.append(o)
    return _wrap(torch.stack(outs) if outs else feat.new_zeros(0, C, ph, pw))


class RoIAlign(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self._output_size, self._spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num, aligned=True):
        return roi_align(x, boxes, boxes_num, self._output_size, self._spatial_scale, aligned=aligned)


class RoIPool(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self._output_size, self._spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return roi_pool(x, boxes, boxes_num, self._output_size, self._spatial_scale)


class PSRoIPool(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return psroi_pool(x, boxes, boxes_num, self.output_size, self.spatial_scale)


# ----------------------------------------------------------------- deformable conv
def deform_conv2d(x, offset, weight, bias=None, stride=1, padding=0, dilation=1, deformable_groups=1, groups=1,
                  mask=None, name=None):
    """Deformable conv v1/v2: every kernel tap is bilinearly sampled at its learned offset
    (batched over the whole output map), then one GEMM per conv group."""
    t, off, w = _u(x), _u(offset), _u(weight)
    st = (stride, stride) if isinstance(stride, int) else tuple(stride)
    pd = (padding, padding) if isinstance(padding, int) else tuple(padding)
    dl = (dilation, dilation) if isinstance(dilation, int) else tuple(dilation)
    N, Cin, H, W = t.shape
    Cout, cin_g, kh, kw = w.shape
    Ho = (H + 2 * pd[0] - dl[0] * (kh - 1) - 1) // st[0] + 1
    Wo = (W + 2 * pd[1] - dl[1] * (kw - 1) - 1) // st[1] + 1
    K = kh * kw
    off = off.view(N, deformable_groups, K, 2, Ho, Wo)
    m = _u(mask).view(N, deformable_groups, K, Ho, Wo) if mask is not None else None
    base_y = (torch.arange(Ho, device=t.device) * st[0] - pd[0]).view(1, Ho, 1).float()
    base_x = (torch.arange(Wo, device=t.device) * st[1] - pd[1]).view(1, 1, Wo).float()
    ky = (torch.arange(kh, device=t.device).repeat_interleave(kw) * dl[0]).view(K, 1, 1).float()
    kx = (torch.arange(kw, device=t.device).repeat(kh) * dl[1]).view(K, 1, 1).float()
    cpg = Cin // deformable_groups
    cols = []
    for n in range(N):
        per_g = []
        for g in range(deformable_groups):
            yy = base_y + ky + off[n, g, :, 0]
            xx = base_x + kx + off[n, g, :, 1]
            v = _bilinear(t[n, g * cpg:(g + 1) * cpg].float(), yy, xx)   # [cpg, K, Ho, Wo]
            if m is not None:
                v = v * m[n, g].unsqueeze(0)
            per_g.append(v)
        cols.append(torch.cat(per_g, 0))                                 # [Cin, K, Ho, Wo]
    col = torch.stack(cols).view(N, groups, cin_g * K, Ho * Wo)
    wg = w.view(groups, Cout // groups, cin_g * K).float()
    out = torch.einsum('gok,ngkp->ngop', wg, col).reshape(N, Cout, Ho, Wo)
    if bias is not None:
        out = out + _u(bias).view(1, -1, 1, 1)
    return _wrap(out.to(t.dtype))


class DeformConv2D(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, deformable_groups=1,
                 groups=1, weight_attr=None, bias_attr=None):
        super().__init__()
        ks = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        fan_in = in_channels // groups * ks[0] * ks[1]
        self.weight = self.create_parameter([out_channels, in_channels // groups, ks[0], ks[1]], attr=weight_attr,
                                            default_initializer=I.Normal(0.0, (2.0 / fan_in) ** 0.5))
        self.bias = None if bias_attr is False else self.create_parameter([out_channels], attr=bias_attr,
                                                                          is_bias=True)
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._deformable_groups, self._groups = deformable_groups, groups

    def forward(self, x, offset, mask=None):
        return deform_conv2d(x, offset, self.weight, self.bias, self._stride, self._padding, self._dilation,
                             self._deformable_groups, self._groups, mask)


# ----------------------------------------------------------------- proposals
def distribute_fpn_proposals(fpn_rois, min_level, max_level, refer_level, refer_scale, pixel_offset=False,
                             rois_num=None, name=None):
    rois = _u(fpn_rois).float()
    off = 1.0 if pixel_offset else 0.0
    w = rois[:, 2] - rois[:, 0] + off
    h = rois[:, 3] - rois[:, 1] + off
    scale = torch.sqrt((w * h).clamp(min=0))
    lvl = torch.floor(torch.log2(scale / refer_scale + 1e-8) + refer_level).clamp(min_level, max_level).long()
    multi, idxs, nums = [], [], []
    bidx = _roi_batch_index(rois_num, rois.shape[0], rois.device) if rois_num is not None else None
    for L in range(min_level, max_level + 1):
        sel = torch.nonzero(lvl == L).squeeze(1)
        multi.append(_wrap(rois[sel]))
        idxs.append(sel)
        if bidx is not None:
            nb = _u(rois_num).numel()
            nums.append(_wrap(torch.bincount(bidx[sel], minlength=nb).to(torch.int32)))
    order = torch.cat(idxs)
    restore = torch.empty_like(order)
    restore[order] = torch.arange(order.numel(), device=order.device)
    return multi, _wrap(restore.view(-1, 1)), (nums if bidx is not None else None)


def generate_proposals(scores, bbox_deltas, img_size, anchors, variances, pre_nms_top_n=6000, post_nms_top_n=1000,
                       nms_thresh=0.5, min_size=0.1, eta=1.0, pixel_offset=False, return_rois_num=False, name=None):
    sc, dl, isz = _u(scores).float(), _u(bbox_deltas).float(), _u(img_size).float()
    an, var = _u(anchors).float().view(-1, 4), _u(variances).float().view(-1, 4)
    N = sc.shape[0]
    off = 1.0 if pixel_offset else 0.0
    all_rois, all_probs, nums = [], [], []
    for n in range(N):
        s = sc[n].permute(1, 2, 0).reshape(-1)
        d = dl[n].permute(1, 2, 0).reshape(-1, 4)
        k = min(pre_nms_top_n, s.numel())
        top = torch.topk(s, k).indices
        s, d, a, v = s[top], d[top], an[top], var[top]
        aw, ah = a[:, 2] - a[:, 0] + off, a[:, 3] - a[:, 1] + off
        ax, ay = a[:, 0] + 0.5 * aw, a[:, 1] + 0.5 * ah
        cx, cy = v[:, 0] * d[:, 0] * aw + ax, v[:, 1] * d[:, 1] * ah + ay
        w = torch.exp(torch.clamp(v[:, 2] * d[:, 2], max=math.log(1000 / 16))) * aw
        h = torch.exp(torch.clamp(v[:, 3] * d[:, 3], max=math.log(1000 / 16))) * ah
        boxes = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - off, cy + h / 2 - off], -1)
        ih, iw = isz[n, 0], isz[n, 1]
        boxes = torch.stack([boxes[:, 0].clamp(0, float(iw) - off), boxes[:, 1].clamp(0, float(ih) - off),
                             boxes[:, 2].clamp(0, float(iw) - off), boxes[:, 3].clamp(0, float(ih) - off)], -1)
        keep = ((boxes[:, 2] - boxes[:, 0] + off) >= min_size) & ((boxes[:, 3] - boxes[:, 1] + off) >= min_size)
        boxes, s = boxes[keep], s[keep]
        k2 = _greedy_nms(boxes, s, nms_thresh)[:post_nms_top_n]
        all_rois.append(boxes[k2])
        all_probs.append(s[k2].view(-1, 1))
        nums.append(k2.numel())
    rois, probs = _wrap(torch.cat(all_rois)), _wrap(torch.cat(all_probs))
    if return_rois_num:
        return rois, probs, _wrap(torch.tensor(nums, dtype=torch.int32))
    return rois, probs, None


def matrix_nms(bboxes, scores, score_threshold, post_threshold, nms_top_k, keep_top_k, use_gaussian=False,
               gaussian_sigma=2.0, background_label=0, normalized=True, return_index=False, return_rois_num=True,
               name=None):
    """Matrix NMS (SOLOv2): scores decayed by the max-IoU compensation matrix, no sequential loop."""
    bb, sc = _u(bboxes).float(), _u(scores).float()     # [N, M, 4], [N, C, M]
    N, C, M = sc.shape
    outs, idxs, nums = [], [], []
    for n in range(N):
        dets = []
        for c in range(C):
            if c == background_label:
                continue
            s = sc[n, c]
            sel = torch.nonzero(s > score_threshold).squeeze(1)
            if sel.numel() == 0:
                continue
            order = sel[torch.argsort(s[sel], descending=True)]
            if nms_top_k > -1:
                order = order[:nms_top_k]
            b = bb[n, order]
            iou = _iou_matrix(b, b).triu(1)
            comp = iou.max(0).values
            if use_gaussian:
                decay = torch.exp(-(iou ** 2 - comp.view(-1, 1) ** 2) / gaussian_sigma).min(0).values
            else:
                decay = ((1 - iou) / (1 - comp.view(-1, 1))).min(0).values
            ds = s[order] * decay
            keep = ds > post_threshold
            for i in torch.nonzero(keep).squeeze(1).tolist():
                dets.append((float(ds[i]), c, order[i].item()))
        dets.sort(key=lambda d: -d[0])
        if keep_top_k > -1:
            dets = dets[:keep_top_k]
        for sv, c, i in dets:
            outs.append(torch.cat([torch.tensor([c, sv], device=bb.device), bb[n, i]]))
            idxs.append(n * M + i)
        nums.append(len(dets))
    out = torch.stack(outs) if outs else bb.new_zeros(0, 6)
    res = [_wrap(out)]
    if return_rois_num:
        res.append(_wrap(torch.tensor(nums, dtype=torch.int32)))
    if return_index:
        res.append(_wrap(torch.tensor(idxs, dtype=torch.long).view(-1, 1)))
    return tuple(res) if len(res) > 1 else res[0]


# ----------------------------------------------------------------- image io
def read_file(filename, name=None):
    with open(filename, 'rb') as f:
        data = f.read()
    return _wrap(torch.frombuffer(bytearray(data), dtype=torch.uint8))


def decode_jpeg(x, mode='unchanged', name=None):
    """JPEG bytes → CHW uint8 (PIL decoder on the host)."""
    import io
    from PIL import Image
    img = Image.open(io.BytesIO(bytes(_u(x).cpu().numpy().tobytes())))
    if mode == 'gray':
        img = img.convert('L')
    elif mode == 'rgb':
        img = img.convert('RGB')
    a = np.array(img)
    t = torch.from_numpy(a)
    t = t.unsqueeze(0) if t.dim() == 2 else t.permute(2, 0, 1)
    return _wrap(t.contiguous())


class ConvNormActivation(Layer):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=None, groups=1, norm_layer=None,
                 activation_layer=None, dilation=1, bias=None):
        super().__init__()
        from .. import nn
        norm_layer = nn.BatchNorm2D if norm_layer is None else norm_layer
        activation_layer = nn.ReLU if activation_layer is None else activation_layer
        if padding is None:
            padding = (kernel_size - 1) // 2 * dilation
        if bias is None:
            bias = norm_layer is None
        layers = [nn.Conv2D(in_channels, out_channels, kernel_size, stride, padding, dilation=dilation,
                            groups=groups, bias_attr=None if bias else False)]
        if norm_layer is not None:
            layers.append(norm_layer(out_channels))
        if activation_layer is not None:
            layers.append(activation_layer())
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        return self.block(x)
