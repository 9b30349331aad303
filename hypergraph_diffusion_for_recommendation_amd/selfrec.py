"""SELFRec's plugin surface, host side: the lifecycle the hot path's callers run in.

The reference's model plugins (``model/graph/<Name>.py``) are constructed by ``SELFRec.execute``
(SELFRec.py:37-42) as ``Name(conf, training_set, test_set, knowledge_set, **kwargs)`` and driven
by ``Recommender.execute`` (base/recommender.py:80-114): build → train → test → evaluate, with
``GraphRecommender`` (base/graph_recommender.py) supplying the data object, the per-epoch
``fast_evaluation`` and the result files. This module is that surface with the same names,
arguments, files and printed measures (paths relative to /root/reference/HD_SELFRec):

* :class:`ModelConf` / :class:`OptionConf` — util/conf.py:11-74 (the ``.conf`` format);
* :func:`default_args` — the argparse defaults of main.py:6-95 as the ``kwargs`` dict;
* :class:`FileIO` — data/loader.py:7-38 (the native multithreaded parser, same line rules);
* :class:`Interaction` — data/ui_graph.py:12-188: the reference's dict maps, built in the same
  first-appearance order, with ``ui_adj`` / ``norm_adj`` / ``interaction_mat`` /
  ``norm_interaction_mat`` built on the device (``ingest.InteractionGraph``) and handed out as
  scipy CSR like the reference's;
* :class:`Recommender`, :class:`GraphRecommender` — the lifecycle, with ``test()`` /
  ``fast_evaluation()`` on the device (batched scores, rated-item masking, ``find_k_largest``
  lists and ranking metrics, ``evaluation.evaluate_test_users``) producing the reference's
  strings bit for bit;
* :func:`early_stopping` — util/evaluation.py:195-202;
* :class:`SELFRec` — SELFRec.py:4-42, resolving ``model.name`` in :data:`PLUGINS`
  (``plugins.PLUGINS``: HCCF, HCCF_diffusion, HGNN_HD4, HGNN_HD3, HGCN, DHCF and the user-row
  sharded HCCF_sharded, HGNN_HD4_sharded, HGNN_HD3_sharded) instead of ``exec`` on
  ``model.<type>.<name>``.

The training loops of the plugins use :func:`sampler.next_batch_pairwise` (bit-identical to
util/sampler.py) and the drop-in encoders; nothing here falls back to the CPU for the path.
"""
from __future__ import annotations

import argparse
import logging
import os
import time
from collections import defaultdict
from os.path import abspath
from typing import Dict, List, Optional

import numpy as np
import torch

from . import evaluation as ev


# ---------------------------------------------------------------------------------------------
# util/conf.py
# ---------------------------------------------------------------------------------------------
def namespace_to_dict(namespace) -> dict:
    """util/conf.py:4-8."""
    return {k: namespace_to_dict(v) if isinstance(v, argparse.Namespace) else v
            for k, v in vars(namespace).items()}


class ModelConf:
    """``key=value`` lines (util/conf.py:11-35): blank lines skipped, a line with more or fewer
    than one '=' reported and skipped, missing keys are fatal on lookup.

    A deliberate restatement of the reference's parser (util/conf.py:10-74, with
    :class:`OptionConf`): ``conf/`` must stay untouched, so the ``.conf`` format has to parse
    byte-identically, quirks included."""

    def __init__(self, file: str):
        self.config: Dict[str, str] = {}
        self.read_configuration(file)

    def __getitem__(self, item):
        if not self.contain(item):
            raise KeyError(f"parameter {item} is not found in the configuration file!")
        return self.config[item]

    def contain(self, key) -> bool:
        return key in self.config

    def read_configuration(self, file: str) -> None:
        if not os.path.exists(file):
            raise IOError(f"config file is not found: {file}")
        with open(file) as f:
            for ind, line in enumerate(f):
                if line.strip() != '':
                    try:
                        key, value = line.strip().split('=')
                        self.config[key] = value
                    except ValueError:
                        print('config file is not in the correct format! Error Line:%d' % ind)


class OptionConf:
    """Space-separated option strings such as ``-topN 10,20`` (util/conf.py:37-74)."""

    def __init__(self, content: str):
        self.line = content.strip().split(' ')
        self.options: Dict[str, object] = {}
        self.mainOption = self.line[0] == 'on'
        for i, item in enumerate(self.line):
            if (item.startswith('-') or item.startswith('--')) and not item[1:].isdigit():
                ind = i + 1
                for j, sub in enumerate(self.line[ind:]):
                    if (sub.startswith('-') or sub.startswith('--')) and not sub[1:].isdigit():
                        ind = j
                        break
                    if j == len(self.line[ind:]) - 1:
                        ind = j + 1
                        break
                try:
                    self.options[item] = ' '.join(self.line[i + 1:i + 1 + ind])
                except IndexError:
                    self.options[item] = 1

    def __getitem__(self, item):
        if not self.contain(item):
            raise KeyError(f"parameter {item} is invalid!")
        return self.options[item]

    def keys(self):
        return self.options.keys()

    def is_main_on(self) -> bool:
        return self.mainOption

    def contain(self, key) -> bool:
        return key in self.options


_MAIN_DEFAULTS = {  # main.py:6-95 (argparse defaults; choices are enforced by main.py itself)
    'experiment': 'full', 'group_id': None, 'missing_pct': None, 'noise_pct': None,
    'model': 'HCCF', 'gpu_id': 0, 'dataset': 'amazon_books', 'seed': 60, 'alpha': 1.0,
    'lrate': 0.001, 'item_ranking': '10,20,40', 'max_epoch': 500, 'batch_size': 4096,
    'hyperedge_num': 32, 'batch_size_kg': 8192, 'n_layers': 2, 'embedding_size': 32,
    'input_dim': 32, 'relation_dim': 32, 'hyper_dim': 32, 'lr_decay': 0.9,
    'weight_decay': 5e-6, 'reg': 0.01, 'reg_kg': 0.01, 'p': 0.3, 'drop_rate': 0.2, 'nheads': 4,
    'temp': 10.0, 'cl_rate': 0.01, 'mode': 'full', 'aug_type': 1,
    'laplacian_type': 'random-walk', 'aggregation_type': 'bi-interaction',
    'conv_dim_list': '[64, 32, 16]', 'mess_dropout': '[0.1, 0.1, 0.1]',
    'early_stopping_steps': 30, 'cf_print_every': 1, 'kg_print_every': 1, 'evaluate_every': 10,
}


def default_args(**overrides) -> dict:
    """The ``kwargs`` dict main.py passes to SELFRec (``namespace_to_dict(parse_arguments())``,
    main.py:128) with its defaults, updated by ``overrides``."""
    unknown = set(overrides) - set(_MAIN_DEFAULTS)
    if unknown:
        raise TypeError(f"default_args: unknown argument(s) {sorted(unknown)}")
    d = dict(_MAIN_DEFAULTS)
    d.update(overrides)
    return d


# ---------------------------------------------------------------------------------------------
# data/loader.py, util/logger.py, util/evaluation.py:195-202
# ---------------------------------------------------------------------------------------------
class FileIO:
    """data/loader.py:7-38."""

    @staticmethod
    def write_file(dir, file, content, op='w'):
        os.makedirs(dir, exist_ok=True)
        with open(dir + file, op) as f:
            f.writelines(content)

    @staticmethod
    def delete_file(file_path):
        if os.path.exists(file_path):
            os.remove(file_path)

    @staticmethod
    def load_data_set(file, rec_type='graph'):
        """[[user, item, 1.0], ...] in file order (header line skipped; ',' or tab separated)
        through the native parser (ingest.load_data_set, same line rules)."""
        from .ingest import load_data_set
        users, items = load_data_set(file)
        return [[u, i, 1.0] for u, i in zip(users.tolist(), items.tolist())]


class Log:
    """util/logger.py:5-17 (./log/<filename>.log)."""

    def __init__(self, module, filename):
        self.logger = logging.getLogger(module)
        self.logger.setLevel(level=logging.INFO)
        os.makedirs('./log/', exist_ok=True)
        handler = logging.FileHandler('./log/' + filename + '.log')
        handler.setFormatter(logging.Formatter(
            '%(asctime)s - %(name)s - %(levelname)s - %(message)s'))
        self.logger.addHandler(handler)

    def add(self, text):
        self.logger.info(text)


def early_stopping(recall_list, stopping_steps):
    """util/evaluation.py:195-202."""
    best_recall = max(recall_list)
    best_step = recall_list.index(best_recall)
    return best_recall, len(recall_list) - best_step - 1 >= stopping_steps


# ---------------------------------------------------------------------------------------------
# data/ui_graph.py
# ---------------------------------------------------------------------------------------------
class Interaction:
    """data/ui_graph.py:12-188: the maps and sets the harness uses, in the reference's
    first-appearance order, and the training matrices (built on the device by
    ``ingest.InteractionGraph``: bit-exact structure and counts, normalised values within 1 ulp
    of scipy/numpy) exposed as scipy CSR like the reference's attributes."""

    def __init__(self, conf, training, test, device=None):
        from .ingest import InteractionGraph
        self.config = conf
        self.training_data = training
        self.test_data = test
        self.user: Dict = {}
        self.item: Dict = {}
        self.id2user: Dict = {}
        self.id2item: Dict = {}
        self.training_set_u = defaultdict(dict)
        self.training_set_i = defaultdict(dict)
        self.test_set = defaultdict(dict)
        self.user_history_dict = defaultdict(dict)
        self.test_set_item = set()
        self.__generate_set()
        self.n_users = len(self.training_set_u)
        self.n_items = len(self.training_set_i)
        self.n_cf_train = len(self.training_data)
        self.n_cf_test = len(self.test_data)
        dev = torch.device(device) if device is not None else torch.device("cuda")
        u = np.fromiter((r[0] for r in training), dtype=np.int64, count=len(training))
        i = np.fromiter((r[1] for r in training), dtype=np.int64, count=len(training))
        self.graph = InteractionGraph(u, i, dev)  # device maps agree with the dicts above
        self.ui_adj = self.graph.to_scipy("ui_adj")
        self.norm_adj = self.graph.to_scipy("norm_adj")
        self.interaction_mat = self.graph.to_scipy("interaction_mat")
        self.inv_interaction_mat = self.interaction_mat.T.tocsr()
        self.norm_interaction_mat = self.graph.to_scipy("norm_interaction_mat")

    def __generate_set(self):  # data/ui_graph.py:43-68
        for entry in self.training_data:
            user, item, rating = entry
            user, item = int(user), int(item)
            if user not in self.user:
                self.user[user] = len(self.user)
                self.id2user[self.user[user]] = user
            if item not in self.item:
                self.item[item] = len(self.item)
                self.id2item[self.item[item]] = item
            if rating == 1.0:
                if user not in self.user_history_dict:
                    self.user_history_dict[user] = []
                self.user_history_dict[user].append(item)
            self.training_set_u[user][item] = rating
            self.training_set_i[item][user] = rating
        for entry in self.test_data:
            user, item, rating = entry
            if user not in self.user:
                continue
            self.test_set[user][item] = rating
            self.test_set_item.add(item)

    def get_user_id(self, u):
        if u in self.user:
            return self.user[u]

    def get_item_id(self, i):
        if i in self.item:
            return self.item[i]

    def training_size(self):
        return len(self.user), len(self.item), len(self.training_data)

    def test_size(self):
        return len(self.test_set), len(self.test_set_item), len(self.test_data)

    def contain(self, u, i):
        return u in self.user and i in self.training_set_u[u]

    def contain_user(self, u):
        return u in self.user

    def contain_item(self, i):
        return i in self.item

    def user_rated(self, u):
        return list(self.training_set_u[u].keys()), list(self.training_set_u[u].values())

    def item_rated(self, i):
        return list(self.training_set_i[i].keys()), list(self.training_set_i[i].values())


# ---------------------------------------------------------------------------------------------
# base/recommender.py, base/graph_recommender.py
# ---------------------------------------------------------------------------------------------
class Recommender:
    """base/recommender.py:9-114."""

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        self.config = conf
        self.experiment = kwargs['experiment']
        self.model_name = self.config['model.name']
        self.ranking = kwargs['item_ranking']
        self.emb_size = int(self.config['embedding.size'])
        self.maxEpoch = int(self.config['num.max.epoch'])
        self.batch_size = int(self.config['batch_size'])
        self.lRate = float(self.config['learnRate'])
        self.lr_decay = float(self.config['learnRateDecay'])
        self.reg = float(self.config['reg.lambda'])
        self.dataset = self.config['dataset']
        self.knowledge = self.config['use.knowledge'] == 'true'
        try:
            self.ss_rate = float(self.config['ss_rate'])
        except (KeyError, ValueError):
            self.ss_rate = 0.0
        current_time = time.strftime("%Y-%m-%d %H-%M-%S", time.localtime(time.time()))
        self.model_log = Log(self.model_name, self.model_name + ' ' + current_time)
        self.result: List[str] = []
        self.recOutput: List[str] = []

    def initializing_log(self):
        self.model_log.add('### model configuration ###')
        for k in self.config.config:
            self.model_log.add(k + '=' + self.config[k])

    def print_model_info(self):
        print('Model:', self.config['model.name'])
        print('Training Set:', abspath(self.config['training.set']))
        print('Test Set:', abspath(self.config['test.set']))
        print('Embedding Dimension:', self.emb_size)
        print('Maximum Epoch:', self.maxEpoch)
        print('Learning Rate:', self.lRate)
        print('Batch Size:', self.batch_size)
        print('Regularization Parameter:', self.reg)

    def build(self):
        pass

    def train(self, load_pretrained=False):
        pass

    def predict(self, u):
        pass

    def test(self):
        pass

    def save(self):
        pass

    def load(self):
        pass

    def evaluate(self, rec_list):
        pass

    def execute(self):
        self.initializing_log()
        self.print_model_info()
        print('Initializing and building model...')
        self.build()
        print('Training Model...')
        self.train(load_pretrained=False)
        print('Testing...')
        rec_list = self.test()
        print('Evaluating...')
        self.evaluate(rec_list)


class GraphRecommender(Recommender):
    """base/graph_recommender.py:18-239 with the evaluation on the device. Plugins set
    ``self.user_emb`` / ``self.item_emb`` (device [U, d] / [I, d]) before ``test`` /
    ``fast_evaluation``, as the reference's do for ``predict``."""

    def __init__(self, conf, training_set, test_set, knowledge_set, **kwargs):
        super().__init__(conf, training_set, test_set, knowledge_set, **kwargs)
        self.device = torch.device(kwargs.get('device') or
                                   f"cuda:{kwargs.get('gpu_id', 0) or 0}")
        self.data = Interaction(conf, training_set, test_set, self.device)
        self.bestPerformance: list = []
        self.topN = [int(num) for num in self.ranking.split(',')]
        self.max_N = max(self.topN)
        exp = kwargs['experiment']
        if exp == 'cold_start':
            exp_name = f"cold_start_{kwargs['group_id']}"
        elif exp == 'missing':
            exp_name = f"missing_{kwargs['missing_pct']}"
        elif exp == 'add_noise':
            exp_name = f"add_noise_{kwargs['noise_pct']}"
        else:
            exp_name = 'full'
        self.output = (f"./results/{self.model_name}/{self.dataset}/{exp_name}/@{self.model_name}"
                       f"-bs:{kwargs['batch_size']}-lr:{kwargs['lrate']}-lrd:{kwargs['lr_decay']}"
                       f"-wdecay:{kwargs['weight_decay']}-reg:{kwargs['reg']}-leaky:{kwargs['p']}"
                       f"-dropout:{kwargs['drop_rate']}-n_layers:{kwargs['n_layers']}"
                       f"-temp:{kwargs['temp']}-cl_rate:{kwargs['cl_rate']}")
        os.makedirs(self.output, exist_ok=True)  # (ranks of a sharded plugin race here)
        self._tests: Optional[ev.TestLists] = None
        self._rated = None

    def print_model_info(self):
        super().print_model_info()
        print('Training Set Size: (user number: %d, item number %d, interaction number: %d)'
              % (self.data.training_size()))
        print('Test Set Size: (user number: %d, item number %d, interaction number: %d)'
              % (self.data.test_size()))
        print('=' * 80)

    def _device_eval(self):
        if self._tests is None:
            self._tests = ev.TestLists(self.data.test_set, self.data.item, self.device)
            self._rated = ev.rated_csr(self.data.interaction_mat, self.device)
        return ev.evaluate_test_users(self.data, self.user_emb, self.item_emb, self.topN,
                                      tests=self._tests, rated=self._rated)

    def test(self) -> Dict:
        """{test user: [(item, score), ...max_N]} in data.test_set order (graph_recommender.py
        :61-92: predict + rated items at -10e8 + find_k_largest), scored on the device."""
        _, ids, sc = self._device_eval()
        ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
        id2item = self.data.id2item
        return {u: [(id2item[int(i)], float(s)) for i, s in zip(ids[r], sc[r])]
                for r, u in enumerate(self._tests.users)}

    def evaluate(self, rec_list):
        """graph_recommender.py:94-119: the recommendation file and the performance file."""
        self.recOutput.append('userId: recommendations in (itemId, ranking score) pairs, * means '
                              'the item is hit.\n')
        for user in self.data.test_set:
            line = str(user) + ':'
            for item in rec_list[user]:
                line += ' (' + str(item[0]) + ',' + str(item[1]) + ')'
                if item[0] in self.data.test_set[user]:
                    line += '*'
            line += '\n'
            self.recOutput.append(line)
        out_dir = self.output + '/'
        FileIO.write_file(out_dir, self.config['model.name'] + '-top-' + str(self.max_N)
                          + 'items' + '.txt', self.recOutput)
        print('The result has been output to ', abspath(out_dir), '.')
        _, ids, _ = self._device_eval()
        self.result = ev.ranking_evaluation(self._tests, ids, self.topN)
        self.model_log.add('###Evaluation Results###')
        self.model_log.add(self.result)
        FileIO.write_file(out_dir, self.config['model.name'] + '-performance' + '.txt',
                          self.result)
        print('The result of %s:\n%s' % (self.model_name, ''.join(self.result)))

    def fast_evaluation(self, epoch, kwargs=None, train_time=None):
        """graph_recommender.py:121-199: device metrics, best-performance bookkeeping (save() on
        improvement), the same printed lines; returns (measure of max_N, data_ep)."""
        print('Evaluating the model...')
        s_test = time.time()
        all_measures, _, _ = self._device_eval()
        e_test = time.time()
        print("Test time: %f s" % (e_test - s_test))
        len_measures = len(self.topN)
        data_ep = {'epoch': epoch, 'train_time': train_time, 'test_time': e_test - s_test}
        for i in range(0, len(all_measures), 5):
            mes = all_measures[i:i + 5]
            topk = int(mes[0].split(' ')[1][:-1])
            data_ep[f'hit@{topk}'] = float(mes[1].split(':')[1][:-1])
            data_ep[f'precision@{topk}'] = float(mes[2].split(':')[1][:-1])
            data_ep[f'recall@{topk}'] = float(mes[3].split(':')[1][:-1])
            data_ep[f'ndcg@{topk}'] = float(mes[4].split(':')[1][:-1])
        measure = all_measures[(len_measures - 1) * 5: (len_measures - 1) * 5 + 5]
        performance = {}
        for m in measure[1:]:
            k, v = m.strip().split(':')
            performance[k] = float(v)
        if len(self.bestPerformance) > 0:
            count = 0
            for k in self.bestPerformance[1]:
                count += 1 if self.bestPerformance[1][k] > performance[k] else -1
            if count < 0:
                self.bestPerformance[1] = performance
                self.bestPerformance[0] = epoch + 1
                self.save()
        else:
            self.bestPerformance.append(epoch + 1)
            self.bestPerformance.append(performance)
            self.save()
        print('-' * 120)
        print('Real-Time Ranking Performance ' + ' (Top-' + str(self.max_N)
              + ' Item Recommendation)')
        measure = [m.strip() for m in measure[1:]]
        print('*Current Performance*')
        print('Epoch:', str(epoch + 1) + ',', '  |  '.join(measure))
        bp = ('Hit Ratio' + ':' + str(self.bestPerformance[1]['Hit Ratio']) + '  |  '
              + 'Precision' + ':' + str(self.bestPerformance[1]['Precision']) + '  |  '
              + 'Recall' + ':' + str(self.bestPerformance[1]['Recall']) + '  |  '
              + 'NDCG' + ':' + str(self.bestPerformance[1]['NDCG']))
        print('*Best Performance* ')
        print('Epoch:', str(self.bestPerformance[0]) + ',', bp)
        print('-' * 120)
        return measure, data_ep

    def save_model(self, model):
        current_time = time.strftime("%Y-%m-%d", time.localtime(time.time()))
        torch.save(model.state_dict(), self.output + '/' + self.config['model.name'] + '@'
                   + current_time + '-weight' + '.pth')

    def save_loss(self, train_losses, rec_losses, reg_losses, cl_losses=None):
        import pandas as pd
        pd.DataFrame(train_losses, columns=['ep', 'loss']).to_csv(self.output + '/train_loss.csv')
        pd.DataFrame(rec_losses, columns=['ep', 'loss']).to_csv(self.output + '/rec_loss.csv')
        pd.DataFrame(reg_losses, columns=['ep', 'loss']).to_csv(self.output + '/reg_loss.csv')
        if cl_losses:
            pd.DataFrame(cl_losses, columns=['ep', 'loss']).to_csv(self.output + '/cl_loss.csv')

    def save_perfomance_training(self, log_train):
        import pandas as pd
        pd.DataFrame(log_train).to_csv(self.output + '/performance.csv')


# ---------------------------------------------------------------------------------------------
# SELFRec.py
# ---------------------------------------------------------------------------------------------
class SELFRec:
    """SELFRec.py:4-42: loads ./dataset/<dataset>/<training.set|test.set> for the 'full'
    experiment (the 'missing' / 'cold_start' / 'add_noise' file layouts likewise) and runs the
    plugin named by ``model.name`` from :data:`plugins.PLUGINS`. The knowledge graph file is
    read only when the configuration enables ``use.knowledge`` (no plugin here uses it)."""

    def __init__(self, config, args=None):
        self.config = config
        self.kwargs = dict(args or {})
        experiment = self.kwargs['experiment']
        root = self.kwargs.get('dataset_root', './dataset')
        ds = config['dataset']
        if experiment == 'full':
            d = f"{root}/{ds}/"
            train, test = d + config['training.set'], d + config['test.set']
        elif experiment == 'missing':
            d = f"{root}/{ds}/{experiment}/"
            pct = self.kwargs['missing_pct']
            train, test = d + f'train_{pct}.txt', d + f'test_{pct}.txt'
        elif experiment == 'cold_start':
            d = f"{root}/{ds}/{experiment}/"
            train, test = d + "train.txt", d + f"test_group_{self.kwargs['group_id']}.txt"
        elif experiment == 'add_noise':
            d = f"{root}/{ds}/{experiment}/"
            pct = self.kwargs['noise_pct']
            train, test = d + f'train_{pct}.txt', d + f'test_{pct}.txt'
        else:
            raise ValueError(f"unknown experiment {experiment!r}")
        self.training_data = FileIO.load_data_set(train, config['model.type'])
        self.test_data = FileIO.load_data_set(test, config['model.type'])
        self.knowledge_data = None
        print('Reading data and preprocessing...')

    def execute(self):
        from .plugins import PLUGINS
        name = self.config['model.name']
        if name not in PLUGINS:
            raise KeyError(f"model {name!r} is not a plugin of this build "
                           f"(available: {sorted(PLUGINS)})")
        kwargs = {k: v for k, v in self.kwargs.items() if k != 'dataset_root'}
        rec = PLUGINS[name](self.config, self.training_data, self.test_data,
                            self.knowledge_data, **kwargs)
        rec.execute()
        return rec
