"""AutoAugment in the GPU train transform (methods/_trainer.py:215-229): the
lc_autoaugment kernel vs the oracle's restatement of torchvision 0.16's ops (oracle.autoaugment),
bit for bit on the uint8 images, for every op of the CIFAR10 / ImageNet / SVHN policies at both
signs and several magnitudes, for random sub-policy draws, and through the whole transform
(augment -> resize -> crop -> flip -> normalise) at the existing transform tolerance.
Parity vs torchvision itself: unpinned (not installed; the oracle restates its published code)."""
import pytest
import torch

from oracle import clip_oracle as o

pytestmark = pytest.mark.gpu

OPS = ["Invert", "Brightness", "Color", "Contrast", "Sharpness", "Posterize", "Solarize",
       "AutoContrast", "Equalize", "ShearX", "ShearY", "TranslateX", "TranslateY", "Rotate"]


def images(n, H, W, seed):
    """ToTensor-valued batches with structure (gradients + noise + flat patches), so equalize,
    autocontrast and the blends see realistic histograms; one constant image (max == min)."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    base = ((xx * 7 + yy * 3) % 256).float().expand(n, 3, H, W).clone()
    noise = torch.randint(-40, 41, (n, 3, H, W), generator=g).float()
    x = (base + noise).clamp(0, 255)
    x[0] = 128.0                      # constant image
    x[1, :, : H // 2] = torch.randint(0, 256, (3, H // 2, W), generator=g).float()
    return x / 255


@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("H,W", [(32, 32), (64, 64)])
def test_autoaug_op_bitexact(dev, op, H, W):
    from lcclip.transforms import augmentation_space, autoaugment
    x = images(5, H, W, seed=len(op) + H)
    mags, signed = augmentation_space(10, H, W)[op]
    bins = [0, 3, 7, 9] if mags.dim() else [None]
    for b in bins:
        base = float(mags[b].item()) if b is not None else 0.0
        for sgn in ((1, -1) if signed else (1,)):
            ops = [(op, base * sgn)]
            got = autoaugment(x.to(dev), ops).cpu()
            ref = o.autoaugment(x, ops)
            assert torch.equal(got, ref), (op, b, sgn, (got - ref).abs().max().item())


@pytest.mark.parametrize("policy", ["cifar10", "imagenet", "svhn"])
def test_autoaug_policy_draws_bitexact(dev, policy):
    """Random sub-policy draws (two ops chained), as TrainTransform draws them."""
    from lcclip.transforms import autoaugment, draw_autoaugment
    gen = torch.Generator().manual_seed(11)
    x = images(8, 32, 32, seed=3)
    seen = set()
    for _ in range(40):
        ops = draw_autoaugment(policy, 32, 32, gen)
        seen.update(op for op, _ in ops)
        got = autoaugment(x.to(dev), ops).cpu()
        assert torch.equal(got, o.autoaugment(x, ops)), ops
    assert len(seen) >= 5


def test_train_transform_with_autoaugment(dev):
    """The whole GPU transform with a drawn sub-policy vs oracle.train_transform(aug_ops=...):
    the augmented uint8 image is exact, the rest at the bounds of test_train_transform_vs_oracle."""
    from lcclip.transforms import TrainTransform
    tf = TrainTransform.for_dataset("cifar100", generator=torch.Generator().manual_seed(2))
    x = images(6, 32, 32, seed=9)
    n_aug = 0
    for _ in range(6):
        ops, i, j, flip = tf.draw(32, 32)
        n_aug += bool(ops)
        ref = o.train_transform(x, 224, 4, i, j, flip, tf.mean, tf.std, aug_ops=ops)
        got = tf(x.to(dev), params=(ops, i, j, flip))
        assert (got.cpu() - ref).abs().max().item() < 2e-6, ops
        pt = tf(x.to(dev), params=(ops, i, j, flip), layout="patches")
        pref = o.patchify(ref, 16)
        assert ((pt.float().cpu() - pref).abs() <= pref.abs() * 2 ** -7 + 1e-6).all()
    assert n_aug >= 3


@pytest.mark.parametrize("op", OPS)
def test_autoaug_op_bitexact_large_image(dev, op):
    """Images larger than the LDS form (ImageNet-R's 3 x 224 x 224; also a ragged 3 x 72 x 90)
    go through lc_autoaugment_ws (working image in HBM) with the same arithmetic: bit-exact vs
    the oracle for every op (these used to be rejected by the kernel)."""
    from lcclip.transforms import augmentation_space, autoaugment
    for (H, W) in ((224, 224), (72, 90)):
        x = images(2, H, W, seed=len(op) + W)
        mags, signed = augmentation_space(10, H, W)[op]
        b = 7 if mags.dim() else None
        base = float(mags[b].item()) if b is not None else 0.0
        for sgn in ((1, -1) if signed else (1,)):
            ops = [(op, base * sgn)]
            got = autoaugment(x.to(dev), ops).cpu()
            ref = o.autoaugment(x, ops)
            assert torch.equal(got, ref), (op, H, W, sgn, (got - ref).abs().max().item())


def test_train_transform_imagenet_r_draws(dev):
    """TrainTransform.for_dataset('imagenet-r') on a 3 x 224 x 224 batch: the ImageNet policy's
    drawn sub-policies (an active op in most draws) run through the whole transform without
    error and match the oracle (the r2 kernel raised LcError on the first active op)."""
    from lcclip.transforms import TrainTransform
    tf = TrainTransform.for_dataset("imagenet-r", generator=torch.Generator().manual_seed(4))
    x = images(3, 224, 224, seed=21)
    n_aug = 0
    for _ in range(5):
        ops, i, j, flip = tf.draw(224, 224)
        n_aug += bool(ops)
        ref = o.train_transform(x, 224, 4, i, j, flip, tf.mean, tf.std, aug_ops=ops)
        got = tf(x.to(dev), params=(ops, i, j, flip))
        assert (got.cpu() - ref).abs().max().item() < 2e-6, ops
    assert n_aug >= 2
