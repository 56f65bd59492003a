#! /usr/bin/env python
"""Drop-in replacement of U2GNN_pytorch/train_pytorch_U2GNN_Sup.py on MI355X.

Same flags (:26-38), seeds (:6,:9), data loading / degree-as-tag rule (:44-56), fold split,
Batch_Loader + neighbour sampling on the global numpy stream (bit-exact input_x, vectorised),
train/evaluate loop, StepLR-on-plateau (:209-210), stdout line (:206-207) and acc file
(<run_folder>/../runs_pytorch_U2GNN_Sup/<model_name>/checkpoints/model_acc.txt, :191-198,212).

Execution: the default trainer is the fused HIP step (u2gnn_hip.train.SupTrainer: kernel loss,
backward into a flat grad buffer, device-side clip + Adam, no per-step host sync except the loss
readout the reference also does).  ``--autograd`` runs the reference's exact loop instead
(model(), cross_entropy, loss.backward(), clip_grad_norm_, torch Adam, StepLR) — on the same kernels.
Extra flags: --precision, --attention, --autograd, --max_steps (0 = full epochs), --world_size /
--dist_backend (data parallelism, u2gnn_hip.cli: one process per GPU, a global step = world_size
consecutive batches of the single stream with the averaged gradient, RCCL all-reduce under the backward).
"""
import math
import os
import sys
import time
from argparse import ArgumentDefaultsHelpFormatter, ArgumentParser

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

torch.manual_seed(123)
np.random.seed(123)

from u2gnn_hip.cli import Run, check_world, self_launch, step_seed  # noqa: E402  (no GPU work at import)

parser = ArgumentParser("U2GNN", formatter_class=ArgumentDefaultsHelpFormatter, conflict_handler='resolve')
parser.add_argument("--run_folder", default="../", help="")
parser.add_argument("--dataset", default="PTC", help="Name of the dataset.")
parser.add_argument("--learning_rate", default=0.0005, type=float, help="Learning rate")
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
parser.add_argument("--autograd", action="store_true", help="reference loop: autograd + torch Adam/StepLR")
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

from pytorch_U2GNN_Sup import TransformerU2GNN, label_smoothing  # noqa: E402
from u2gnn_hip.batching import BatchLoader, GraphStore  # noqa: E402
from u2gnn_hip.core import DeviceBatch  # noqa: E402
from u2gnn_hip.dp import GradAllReduce, OverlappedGradAllReduce, broadcast_params  # noqa: E402
from u2gnn_hip.train import SupTrainer  # noqa: E402
from util import load_data, separate_data  # noqa: E402

if not torch.cuda.is_available():
    raise SystemExit("train_pytorch_U2GNN_Sup: the MI355X path needs a GPU (no CPU fallback)")
run = Run.init(args.dist_backend)
check_world(run.world, args.world_size)   # default 1: the launcher's WORLD_SIZE
device = run.device()
torch.cuda.set_device(device)
torch.cuda.manual_seed_all(123)
log = print if run.main else (lambda *a, **k: None)   # rank 0 prints and writes the acc file

log(args)
log("Loading data...")
use_degree_as_tag = args.dataset in ('COLLAB', 'IMDBBINARY', 'IMDBMULTI')
graphs, num_classes = load_data(args.dataset, use_degree_as_tag)
train_graphs, test_graphs = separate_data(graphs, args.fold_idx)
feature_dim_size = graphs[0].node_features.shape[1]
log(feature_dim_size)
reddit = "REDDIT" in args.dataset
if reddit:
    feature_dim_size = 4
train_store = GraphStore(train_graphs, reddit_tile=4 if reddit else 0)
test_store = GraphStore(test_graphs, reddit_tile=4 if reddit else 0)
# native assembly; node features gathered on the GPU from a device-resident copy (DeviceBatch.from_store)
batch_nodes = BatchLoader(train_store, args.batch_size, args.num_neighbors, gather_x=False)
log("Loading data... finished!")

model = TransformerU2GNN(feature_dim_size=feature_dim_size, ff_hidden_size=args.ff_hidden_size,
                         num_classes=num_classes, dropout=args.dropout, num_self_att_layers=args.num_timesteps,
                         num_U2GNN_layers=args.num_hidden_layers, precision=args.precision,
                         attention=args.attention).to(device)
num_batches_per_epoch = int((len(train_graphs) - 1) / args.batch_size) + 1
# global steps per epoch: each consumes world_size batches of the stream
steps_per_epoch = -(-num_batches_per_epoch // run.world)


train_X = torch.from_numpy(train_store.X).to(device)


def to_device(hb):
    if hb.X_concat is None:
        return DeviceBatch.from_store(hb, train_X, device=device)
    return DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat, hb.labels, device=device)


def cross_entropy(pred, soft_targets):
    logsoftmax = nn.LogSoftmax(dim=1)
    return torch.mean(torch.sum(- soft_targets * logsoftmax(pred), 1))


if args.autograd:
    for p in model.parameters():   # every rank starts from rank 0's weights (identical under the seed anyway)
        run.broadcast(p.data)
    if run.world > 1:   # the module draws its dropout seeds from torch's generator: one stream per rank
        torch.manual_seed(123 + run.rank)
    optimizer = torch.optim.Adam(model.parameters(), lr=args.learning_rate)
    scheduler = torch.optim.lr_scheduler.StepLR(optimizer, step_size=num_batches_per_epoch, gamma=0.1)
    trainer = None
else:
    trainer = SupTrainer(model, lr=args.learning_rate, max_norm=0.5)
    if run.world > 1:
        broadcast_params(trainer.flat)
        if args.dist_backend == "nccl":   # per-layer all-reduce on RCCL's stream under the backward
            ar = OverlappedGradAllReduce(trainer.flat)
            model.core.stack.grad_ready = ar.layer_done
            trainer.grad_sync = ar
        else:                              # gloo: bucketed, after the backward
            trainer.grad_sync = GradAllReduce(bucket_mb=8.0)
    sched_steps = 0
steps_done = 0


def train():
    """One epoch (train_pytorch_U2GNN_Sup.py:149-164); returns the sum of the batches' losses (all ranks')."""
    global steps_done
    model.train()
    total_loss = 0.
    acc = torch.zeros(1, device=device)   # data parallel: the ranks' losses, summed once per epoch
    for _ in range(steps_per_epoch):
        if args.max_steps and steps_done >= args.max_steps:
            break
        hb, index = run.next_batch(batch_nodes)   # this rank's batch of the next global step
        b = to_device(hb)
        if args.autograd:
            optimizer.zero_grad()
            prediction_scores = model(b, None, None)
            loss = cross_entropy(prediction_scores, label_smoothing(b.labels, num_classes))
            loss.backward()
            run.average_grads(model.parameters())
            torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
            optimizer.step()
        else:
            loss = trainer.step(b, seed=step_seed(123, index))
        if run.world > 1:
            acc += loss.detach()
        else:
            total_loss += loss.item()
        steps_done += 1
    return run.sum(acc) if run.world > 1 else total_loss


def evaluate():
    model.eval()
    with torch.no_grad():
        prediction_output = []
        idx = np.arange(len(test_graphs))
        for i in range(0, len(test_graphs), args.batch_size):
            sampled_idx = idx[i:i + args.batch_size]
            if len(sampled_idx) == 0:
                continue
            # same numpy draws as the reference's get_batch_data on the test graphs (:178)
            hb = test_store.assemble(sampled_idx, args.num_neighbors)
            prediction_output.append(model(to_device(hb), None, None).detach())
    prediction_output = torch.cat(prediction_output, 0)
    predictions = prediction_output.max(1, keepdim=True)[1]
    labels = torch.LongTensor([graph.label for graph in test_graphs]).to(device)
    correct = predictions.eq(labels.view_as(predictions)).sum().cpu().item()
    return correct / float(len(test_graphs))


out_dir = os.path.abspath(os.path.join(args.run_folder, "../runs_pytorch_U2GNN_Sup", args.model_name))
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
    acc_test = evaluate()
    log('| epoch {:3d} | time: {:5.2f}s | loss {:5.2f} | test acc {:5.2f} | '.format(
        epoch, (time.time() - epoch_start_time), train_loss, acc_test * 100))
    if epoch > 5 and cost_loss[-1] > np.mean(cost_loss[-6:-1]):
        if args.autograd:
            scheduler.step()
        else:   # StepLR(step_size=num_batches_per_epoch, gamma=0.1) stepped on plateau only
            sched_steps += 1
            trainer.set_lr(args.learning_rate * 0.1 ** (sched_steps // num_batches_per_epoch))
    if write_acc is not None:
        write_acc.write('epoch ' + str(epoch) + ' fold ' + str(args.fold_idx) + ' acc ' + str(acc_test * 100) + '%\n')
    if args.max_steps and steps_done >= args.max_steps:
        break

if write_acc is not None:
    write_acc.close()
if os.environ.get("U2GNN_PARAM_CHECKSUM"):   # tests: every rank's final parameters
    sys.stderr.write("param_checksum rank %d %.10e %.10e\n" % (run.rank, sum(float(p.double().sum()) for p in model.parameters()),
                                                            sum(float(p.double().abs().sum()) for p in model.parameters())))
run.close()
