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
--eval_every (0 = evaluate every epoch like the reference).
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

from pytorch_U2GNN_UnSup import TransformerU2GNN  # noqa: E402
from u2gnn_hip.batching import BatchLoader, GraphStore  # noqa: E402
from u2gnn_hip.core import DeviceBatch  # noqa: E402
from u2gnn_hip.unsup import UnSupTrainer, fold_accuracies, graph_embeddings  # noqa: E402
from util import load_data, separate_data_idx  # noqa: E402

if not torch.cuda.is_available():
    raise SystemExit("train_pytorch_U2GNN_UnSup: the MI355X path needs a GPU (no CPU fallback)")
device = torch.device("cuda")
print("using device {} for pytorch computation".format(device))
torch.cuda.manual_seed_all(123)

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
parser.add_argument("--precision", default="fp32", choices=["fp32", "bf16x3", "mixed", "bf16"],
                    help="matrix-core precision (MI355X): fp32 exact, bf16x3 split-bf16 (~fp32), mixed (bf16x3 "
                         "with the attention-backward dS/dQ/dK products in bf16), bf16")
parser.add_argument("--attention", default="nodes", choices=["nodes", "neighbors"],
                    help="nodes = the fork's attention over all nodes of the batch; neighbors = the paper's "
                         "attention over each node's k+1 sampled neighbours")
parser.add_argument("--max_steps", default=0, type=int, help="stop after this many train steps (0 = no limit)")
args = parser.parse_args()

print(args)
print("Loading data...")
use_degree_as_tag = args.dataset in ('COLLAB', 'IMDBBINARY', 'IMDBMULTI')
graphs, num_classes = load_data(args.dataset, use_degree_as_tag)
graph_labels = np.array([graph.label for graph in graphs])
feature_dim_size = graphs[0].node_features.shape[1]
print(feature_dim_size)
reddit = "REDDIT" in args.dataset
if reddit:
    feature_dim_size = 4
store = GraphStore(graphs, reddit_tile=4 if reddit else 0)
store_X = torch.from_numpy(store.X).to(device)
vocab_size = int(store.node_start[-1])
# native assembly; node features gathered on the GPU from a device-resident copy (DeviceBatch.from_store)
batch_nodes = BatchLoader(store, args.batch_size, args.num_neighbors, with_input_y=True, gather_x=False)
print("Loading data... finished!")

model = TransformerU2GNN(feature_dim_size=feature_dim_size, ff_hidden_size=args.ff_hidden_size,
                         dropout=args.dropout, num_self_att_layers=args.num_timesteps,
                         vocab_size=vocab_size, sampled_num=args.sampled_num,
                         num_U2GNN_layers=args.num_hidden_layers, device=device, precision=args.precision,
                         attention=args.attention).to(device)
trainer = UnSupTrainer(model, lr=args.learning_rate, max_norm=0.5)
num_batches_per_epoch = int((len(graphs) - 1) / args.batch_size) + 1
sched_steps = 0
steps_done = 0


def train():
    global steps_done
    model.train()
    total_loss = 0.
    for _ in range(num_batches_per_epoch):
        if args.max_steps and steps_done >= args.max_steps:
            break
        hb = batch_nodes()
        b = DeviceBatch.from_store(hb, store_X, device=device)
        sid = torch.from_numpy(model.ss.draw_samples()).to(device)
        total_loss += trainer.step(b, sid).item()
        steps_done += 1
    return total_loss


FOLDS = [separate_data_idx(graphs, fold_idx) for fold_idx in range(10)]


def evaluate():
    model.eval()
    with torch.no_grad():
        emb = graph_embeddings(model.ss.weight.detach(), store.node_start).cpu().numpy()
    acc_10folds = fold_accuracies(emb, graph_labels, FOLDS)
    for fold_idx, ACC in enumerate(acc_10folds):
        print('epoch ', epoch, ' fold ', fold_idx, ' acc ', ACC)
    return statistics.mean(acc_10folds), statistics.stdev(acc_10folds)


out_dir = os.path.abspath(os.path.join(args.run_folder, "../runs_pytorch_U2GNN_UnSup", args.model_name))
print("Writing to {}\n".format(out_dir))
checkpoint_dir = os.path.abspath(os.path.join(out_dir, "checkpoints"))
checkpoint_prefix = os.path.join(checkpoint_dir, "model")
os.makedirs(checkpoint_dir, exist_ok=True)
write_acc = open(checkpoint_prefix + '_acc.txt', 'w')

cost_loss = []
for epoch in range(1, args.num_epochs + 1):
    epoch_start_time = time.time()
    train_loss = train()
    cost_loss.append(train_loss)
    mean_10folds, std_10folds = evaluate()
    print('| epoch {:3d} | time: {:5.2f}s | loss {:5.2f} | mean {:5.2f} | std {:5.2f} | '.format(
        epoch, (time.time() - epoch_start_time), train_loss, mean_10folds * 100, std_10folds * 100))
    if epoch > 5 and cost_loss[-1] > np.mean(cost_loss[-6:-1]):
        sched_steps += 1
        trainer.opt.set_lr(args.learning_rate * 0.1 ** (sched_steps // num_batches_per_epoch))
    write_acc.write('epoch ' + str(epoch) + ' mean: ' + str(mean_10folds * 100) + ' std: ' + str(std_10folds * 100) + '\n')
    if args.max_steps and steps_done >= args.max_steps:
        break

write_acc.close()
