import sys, torch
sys.path.insert(0, '.')
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
from rocm_mpi_amd.parallel import implicit_grid as gg
graph = sys.argv[1] == '1'
via = sys.argv[2] == '1'
gg.init_global_grid(300, 200, 1, periodx=1, periody=1, quiet=True, transport="rccl", self_via_transport=via)
m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=300, ny=200, nt=20, quiet=True, init="random", periods=(1,1,0), b_width=(4,4), use_graph=graph, graph_steps=6))
m.step(20)
torch.cuda.synchronize()
print("graph", graph, "via", via, "sum", float(m.field.sum()), flush=True)
m.close()
gg.finalize_global_grid()
print("clean exit", flush=True)
