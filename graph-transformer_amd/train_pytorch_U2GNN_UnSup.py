#! /usr/bin/env python
"""Drop-in replacement of U2GNN_pytorch/train_pytorch_U2GNN_UnSup.py on MI355X.

Same flags (:29-41, lr default 0.005), seeds, data loading, vocabulary = all nodes of the dataset
(graph_pool over all graphs, :92-94), Batch_Loader over all graphs with input_y = the batch's
global node ids (:96-134), loss = sum of the sampled-softmax losses (:156), clip 0.5 + Adam,
StepLR-on-plateau, evaluation = graph embeddings spmm(graph_pool, ss.weight) + 10-fold
LogisticRegression(liblinear, tol=1e-3) (:164-188), stdout line (:207) and acc file
(<run_folder>/../runs_pytorch_U2GNN_UnSup/<model_name>/checkpoints/model_acc.txt).

The fork's file cannot run as shipped; this runs its working semantics
(pytorch_U2GNN_UnSup.TransformerU2GNN of this package).  Extra flags: --precision, --attention, --max_steps,
--world_size / --dist_backend (data parallelism, u2gnn_hip.cli: rank r trains batch r of each global step
with the r-th sample draw of the step; encoder gradients all-reduced, the touched ss.weight rows
all-gathered, dp.UnSupGradSync).
"""
import os
import statistics
import sys
import time
from argparse import ArgumentDefaultsHelpFormatter, ArgumentParser

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.manual_seed(123)
np.random.seed(123)

from u2gnn_hip.cli import Run, check_world, self_launch, step_seed  # noqa: E402  (no GPU work at import)

parser = ArgumentParser("U2GNN", formatter_class=ArgumentDefaultsHelpFormatter, conflict_handler='resolve')
parser.add_argument("--run_folder", default="../", help="")
parser.add_argument("--dataset", default="PTC", help="Name of the dataset.")
parser.add_argument("--learning_rate", default=0.005, type=float, help="Learning rate")
parser.add_argument("--batch_size", default=4, type=int, help="Batch Size")
parser.add_argument("--num_epochs", default=50, type=int, help="Number of training epochs")
parser.add_argument("--model_name", default='PTC', help="")
parser.add_argument('--sampled_num', default=512, type=int, help='')
parser.add_argument("--dropout", default=0.5, type=float, help="")
parser.add_argument("--num_hidden_layers", default=1, type=int, help="")
parser.add_argument("--num_timesteps", default=1, type=int, help="Timestep T ~ Number of self-attention layers within each U2GNN layer")
parser.add_argument("--ff_hidden_size", default=1024, type=int, help="The hidden size for the feedforward layer")
parser.add_argument("--num_neighbors", default=4, type=int, help="")
parser.add_argument('--fold_idx', type=int, default=1, help='The fold index. 0-9.')
parser.add_argument("--precision", default="fp32", choices=["fp32", "bf16x3", "mixed", "bf16", "fwd32", "fwd6", "fwdh"],
                    help="matrix-core precision (MI355X): fp32 exact, bf16x3 split-bf16 (~fp32), mixed (bf16x3 "
                         "with the attention-backward dS/dQ/dK products in bf16), bf16")
parser.add_argument("--attention", default="nodes", choices=["nodes", "neighbors"],
                    help="nodes = the fork's attention over all nodes of the batch; neighbors = the paper's "
                         "attention over each node's k+1 sampled neighbours")
parser.add_argument("--max_steps", default=0, type=int, help="stop after this many train steps (0 = no limit)")
parser.add_argument("--world_size", default=1, type=int,
                    help="data-parallel ranks, one per GPU (started here under torch.distributed.run unless a "
                         "launcher already set WORLD_SIZE; left at 1 under a launcher it takes WORLD_SIZE).  "
                         "Epochs round up to a multiple of world_size batches (u2gnn_hip/cli.py)")
parser.add_argument("--dist_backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend: nccl = RCCL over xGMI; gloo = several ranks on one GPU (tests)")
args = parser.parse_args()

_rc = self_launch(args.world_size, __file__, sys.argv[1:])   # before anything touches the GPU
if _rc is not None:
    sys.exit(_rc)

from pytorch_U2GNN_UnSup import TransformerU2GNN  # noqa: E402
from u2gnn_hip.batching import BatchLoader, GraphStore  # noqa: E402
from u2gnn_hip.core import DeviceBatch  # noqa: E402
from u2gnn_hip.dp import UnSupGradSync, broadcast_params, max_batch_nodes  # noqa: E402
from u2gnn_hip.unsup import UnSupTrainer, fold_accuracies, graph_embeddings  # noqa: E402
from util import load_data, separate_data_idx  # noqa: E402

if not torch.cuda.is_available():
    raise SystemExit("train_pytorch_U2GNN_UnSup: the MI355X path needs a GPU (no CPU fallback)")
run = Run.init(args.dist_backend)
check_world(run.world, args.world_size)   # default 1: the launcher's WORLD_SIZE
device = run.device()
torch.cuda.set_device(device)
log = print if run.main else (lambda *a, **k: None)   # rank 0 prints and writes the acc file
log("using device {} for pytorch computation".format(device))
torch.cuda.manual_seed_all(123)

log(args)
log("Loading data...")
use_degree_as_tag = args.dataset in ('COLLAB', 'IMDBBINARY', 'IMDBMULTI')
graphs, num_classes = load_data(args.dataset, use_degree_as_tag)
graph_labels = np.array([graph.label for graph in graphs])
feature_dim_size = graphs[0].node_features.shape[1]
log(feature_dim_size)
reddit = "REDDIT" in args.dataset
if reddit:
    feature_dim_size = 4
store = GraphStore(graphs, reddit_tile=4 if reddit else 0)
store_X = torch.from_numpy(store.X).to(device)
vocab_size = int(store.node_start[-1])
# native assembly; node features gathered on the GPU from a device-resident copy (DeviceBatch.from_store)
batch_nodes = BatchLoader(store, args.batch_size, args.num_neighbors, with_input_y=True, gather_x=False)
log("Loading data... finished!")

model = TransformerU2GNN(feature_dim_size=feature_dim_size, ff_hidden_size=args.ff_hidden_size,
                         dropout=args.dropout, num_self_att_layers=args.num_timesteps,
                         vocab_size=vocab_size, sampled_num=args.sampled_num,
                         num_U2GNN_layers=args.num_hidden_layers, device=device, precision=args.precision,
                         attention=args.attention).to(device)
trainer = UnSupTrainer(model, lr=args.learning_rate, max_norm=0.5)
if run.world > 1:
    broadcast_params(trainer.flat)
    sync = UnSupGradSync(trainer.flat, max_batch_nodes(store.node_start, args.batch_size))
    trainer.grad_sync = trainer.row_sync = sync
num_batches_per_epoch = int((len(graphs) - 1) / args.batch_size) + 1
# global steps per epoch: each consumes world_size batches of the stream
steps_per_epoch = -(-num_batches_per_epoch // run.world)
sched_steps = 0
steps_done = 0


def train():
    """One epoch (train_pytorch_U2GNN_UnSup.py:149-162); returns the sum of the batches' losses (all ranks')."""
    global steps_done
    model.train()
    total_loss = 0.
    acc = torch.zeros(1, device=device)   # data parallel: the ranks' losses, summed once per epoch
    for _ in range(steps_per_epoch):
        if args.max_steps and steps_done >= args.max_steps:
            break
        hb, index = run.next_batch(batch_nodes)   # this rank's batch of the next global step
        b = DeviceBatch.from_store(hb, store_X, device=device)
        # one sample draw per batch of the stream, in stream order (the sampler is replicated on every rank)
        draws = [model.ss.draw_samples() for _ in range(run.world)]
        sid = torch.from_numpy(draws[run.rank]).to(device)
        loss = trainer.step(b, sid, seed=step_seed(123, index))
        if run.world > 1:
            acc += loss.detach()
        else:
            total_loss += loss.item()
        steps_done += 1
    return run.sum(acc) if run.world > 1 else total_loss


FOLDS = [separate_data_idx(graphs, fold_idx) for fold_idx in range(10)]


def evaluate():
    model.eval()
    with torch.no_grad():
        emb = graph_embeddings(model.ss.weight.detach(), store.node_start).cpu().numpy()
    acc_10folds = fold_accuracies(emb, graph_labels, FOLDS)
    for fold_idx, ACC in enumerate(acc_10folds):
        log('epoch ', epoch, ' fold ', fold_idx, ' acc ', ACC)
    return statistics.mean(acc_10folds), statistics.stdev(acc_10folds)


out_dir = os.path.abspath(os.path.join(args.run_folder, "../runs_pytorch_U2GNN_UnSup", args.model_name))
log("Writing to {}\n".format(out_dir))
checkpoint_dir = os.path.abspath(os.path.join(out_dir, "checkpoints"))
checkpoint_prefix = os.path.join(checkpoint_dir, "model")
if run.main:
    os.makedirs(checkpoint_dir, exist_ok=True)
write_acc = open(checkpoint_prefix + '_acc.txt', 'w') if run.main else None

cost_loss = []
for epoch in range(1, args.num_epochs + 1):
    epoch_start_time = time.time()
    train_loss = train()
    cost_loss.append(train_loss)
    mean_10folds, std_10folds = evaluate()
    log('| epoch {:3d} | time: {:5.2f}s | loss {:5.2f} | mean {:5.2f} | std {:5.2f} | '.format(
        epoch, (time.time() - epoch_start_time), train_loss, mean_10folds * 100, std_10folds * 100))
    if epoch > 5 and cost_loss[-1] > np.mean(cost_loss[-6:-1]):
        sched_steps += 1
        trainer.opt.set_lr(args.learning_rate * 0.1 ** (sched_steps // num_batches_per_epoch))
    if write_acc is not None:
        write_acc.write('epoch ' + str(epoch) + ' mean: ' + str(mean_10folds * 100) + ' std: ' + str(std_10folds * 100) + '\n')
    if args.max_steps and steps_done >= args.max_steps:
        break

if write_acc is not None:
    write_acc.close()
if os.environ.get("U2GNN_PARAM_CHECKSUM"):   # tests: every rank's final parameters
    sys.stderr.write("param_checksum rank %d %.10e %.10e\n" % (run.rank, sum(float(p.double().sum()) for p in model.parameters()),
                                                            sum(float(p.double().abs().sum()) for p in model.parameters())))
run.close()
