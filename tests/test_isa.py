"""ISA checks of hand-counted memory waits (CPU: hipcc cross-compiles the device code to gfx950
assembly; no GPU needed).

adapter_ln_fwd_kernel (peft.hip) waits at the top of each 16-row block with a COUNTED
`s_waitcnt vmcnt(tail)`: the previous block's stores may stay in flight while the block's
LDS-DMAs must have landed. CDNA retires vector-memory ops in issue order, so the count is right
only while the loop issues exactly `tail` stores after its last LDS-DMA — NST + 3 on the waves
that store everything: the h block (16 B), mean and rstd (4 B each), then x_out and y as whole-row
1-KiB pieces through buffer descriptors (NST = 2 D / 256 + D / 256 per wave, D / 256 + D / 256
with the half residual stream; hipcc rotates the
loop, so those appear above the loop header in the text). Fewer stores emitted (e.g. two merged)
would let a read of a slot whose DMA has not landed through, silently; more would only make the
wait conservative. This test pins the emitted count to the one the kernel source assumes
(ADVICE r3)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lifelong-clip_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def peft_asm(tmp_path_factory):
    if not os.path.exists(HIPCC) or shutil.which("make") is None:
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "peft.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17",
                    f"-I{os.path.join(ROOT, 'include')}", "--cuda-device-only", "-S",
                    os.path.join(CSRC, "peft.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    return out.read_text()


def function_body(asm, pattern):
    m = re.search(r"^(" + pattern + r"[^:\s]*):", asm, re.M)
    assert m, f"kernel {pattern} not found in the assembly"
    start = m.end()
    end = asm.index(".Lfunc_end", start)
    return asm[start:end]


@pytest.mark.parametrize("D", [768, 512])
@pytest.mark.parametrize("xt", ["f", "DF16_"])
def test_adapter_ln_fwd_store_tail_matches_wait(peft_asm, D, xt):
    """xt: the residual element type (f32, or IEEE half: x_out is then D / 256 pieces per wave
    instead of 2 D / 256)."""
    body = function_body(peft_asm, rf"_ZN12_GLOBAL__N_121adapter_ln_fwd_kernelILi{D}E{xt}E")
    lines = [ln.strip() for ln in body.splitlines()]
    dma = [i for i, ln in enumerate(lines) if ln.startswith("global_load_lds") or
           (ln.startswith("buffer_load") and " lds" in ln)]
    assert dma, "no LDS-DMA in the kernel"
    tail = [ln.split()[0] for ln in lines[dma[-1] + 1:]
            if ln.startswith(("global_store", "buffer_store"))]
    NST = (2 * D // 256 if xt == "f" else D // 256) + D // 256
    # h block (16 B, waves 0-1), mean / rstd (wave 0) after the last DMA in the text
    assert tail.count("global_store_dwordx4") == 1, tail
    assert tail.count("global_store_dword") == 2, tail
    # the whole-row x_out / y pieces: the kernel's only buffer stores
    pieces = [ln for ln in lines if ln.startswith("buffer_store")]
    assert len(pieces) == NST and all(p.startswith("buffer_store_dwordx4") for p in pieces), pieces
    # and the counted waits the source derives from it are the ones emitted
    waits = {int(x) for x in re.findall(r"s_waitcnt vmcnt\((\d+)\)", body)}
    assert {NST, NST + 1, NST + 3} <= waits, sorted(waits)


@pytest.fixture(scope="module")
def gemm_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "gemm.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17",
                    f"-I{os.path.join(ROOT, 'include')}", "--cuda-device-only", "-S",
                    os.path.join(CSRC, "gemm.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    return out.read_text()


def test_gemm_kernels_keep_registers(gemm_asm):
    """The 256x256 GEMM kernels run at the register-file limit (gemm8: 256 VGPRs per wave at two
    waves per SIMD; the 4-wave kernel: 256 VGPRs + 256 AGPRs): an edit that makes hipcc spill
    costs 30-70 % on the step shapes without changing a result (r4: a tile loop added to gemm8
    spilled 312-696 B per lane; fc2 dX 265 -> 459 us). Every instantiation must keep
    ScratchSize 0, and the 4-wave kernel's main loop must keep its accumulators in AGPRs (no
    v_accvgpr copies between MFMAs).
    The stream-K / row-panel instantiations (gemm8_kernel<EPI, false, true>: non-default A/B
    schedules, lc_gemm_set_streamk) loop over tile segments; they may spill at the segment
    boundaries (156 B, a few scratch accesses per segment), but not inside the k-tile loop."""
    found = 0
    for m in re.finditer(r"^(_ZN12_GLOBAL__N_1\d+(gemm8_kernel|gemm_w4_kernel|gemm_pp_kernel)"
                         r"I\w+?EE\w*):", gemm_asm, re.M):
        end = gemm_asm.index(".Lfunc_end", m.end())
        tail = gemm_asm[end:end + 4000]
        scratch = re.search(r"; ScratchSize: (\d+)", tail)
        assert scratch, m.group(1)
        if re.match(r"_ZN12_GLOBAL__N_112gemm8_kernelILi\d+ELb0ELb1EE", m.group(1)):
            for loop in k_loops(gemm_asm[m.end():end]):
                assert "scratch_" not in loop, f"{m.group(1)}: scratch access in the k-tile loop"
        else:
            assert int(scratch.group(1)) == 0, f"{m.group(1)} spills: {scratch.group(0)}"
        found += 1
    assert found >= 20, found


def k_loops(body):
    """The MFMA loops of a kernel body: blocks from a label to a backward branch to it that
    contain at least 32 MFMAs and no other loop's label nested deeper than 600 lines."""
    lines = body.splitlines()
    labels = {}
    for i, ln in enumerate(lines):
        mm = re.match(r"^(\.LBB\d+_\d+):", ln.strip())
        if mm:
            labels[mm.group(1)] = i
    out = []
    for i, ln in enumerate(lines):
        t = ln.strip()
        if t.startswith(("s_cbranch", "s_branch")):
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] < i and i - labels[tgt] < 600:
                seg = "\n".join(lines[labels[tgt]:i + 1])
                if seg.count("v_mfma") >= 32:
                    out.append(seg)
    assert out, "no k-tile loop found"
    return out


def test_peft_walkers_do_not_spill(peft_asm):
    """The persistent adapter walkers (adapter_ln_fwd_kernel, adapter_bwd_fused_kernel) count
    their vector-memory operations by hand in `s_waitcnt vmcnt(n)`. A register spill adds scratch
    loads and stores to that count. Its reloads also wait vmcnt(0) and drain the DMAs in flight.
    (r4: a variant with contiguous per-walker row shares spilled 4 B per lane in
    adapter_ln_fwd<768> — hoisted per-lane DMA addresses — until its DMA lambdas recomputed their
    lane terms.) Every instantiation keeps ScratchSize 0: adapter_ln_fwd (4), adapter_bwd_fused
    <12|8, dz> (2) and its half-gradient forms <12|8, dz|dpre only, g16> (4)."""
    found = 0
    for m in re.finditer(r"^(_ZN12_GLOBAL__N_1\d+(adapter_ln_fwd_kernel|adapter_bwd_fused_kernel)"
                         r"I\w+?EE\w*):", peft_asm, re.M):
        end = peft_asm.index(".Lfunc_end", m.end())
        scratch = re.search(r"; ScratchSize: (\d+)", peft_asm[end:end + 4000])
        assert scratch and int(scratch.group(1)) == 0, f"{m.group(1)} spills: {scratch.group(0)}"
        found += 1
    assert found == 10, found
