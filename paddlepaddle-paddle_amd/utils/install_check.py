"""paddle.utils.run_check (reference: python/paddle/utils/install_check.py)."""


def run_check():
    import torch
    import paddle
    print(f"Running verify PaddlePaddle(MI355X) program ... version {paddle.__version__}")
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    dev = 'gpu:0' if n else 'cpu'
    paddle.set_device(dev)
    net = paddle.nn.Linear(16, 4)
    opt = paddle.optimizer.SGD(0.01, parameters=net.parameters())
    loss = net(paddle.randn([8, 16])).mean()
    loss.backward()
    opt.step()
    if n:
        from paddle import ops
        x = paddle.randn([64, 256]).astype('bfloat16')
        ln = paddle.nn.LayerNorm(256)
        ln.to(dtype='bfloat16')
        ln(x)
        ok = ops.native_loaded()
        print(f"HIP kernel library loaded: {ok}; devices: {n} x {torch.cuda.get_device_name(0)}")
        print(f"PaddlePaddle works well on {n} GPU{'s' if n > 1 else ''}.")
    else:
        print("PaddlePaddle works well on CPU.")
    print("PaddlePaddle is installed successfully! Let's start deep learning with PaddlePaddle now.")
