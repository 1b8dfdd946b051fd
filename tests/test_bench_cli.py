"""bench.py argument contract (the driver runs `bench.py --gpus N --steps K --warmup W`,
N > 1 under torch.distributed.run): the batch is resolved before either path runs."""
import bench


def test_default_is_config2_batch256():
    a = bench.parse_args([])
    assert (a.config, a.batch, a.gpus) == (2, 256, 1)


def test_driver_multi_gpu_args_resolve_batch():
    a = bench.parse_args(["--gpus", "8", "--steps", "50", "--warmup", "10"])
    assert a.batch == 256 and a.steps == 50 and a.warmup == 10


def test_config3_batch4096():
    assert bench.parse_args(["--config", "3"]).batch == 4096
