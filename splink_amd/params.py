"""Model state (reference: splink/params.py).

`Params.params` has the reference's exact layout -- {"λ": float, "π": {"gamma_<col>": {...,
"prob_dist_match": {"level_<i>": {"value": i, "probability": p}}, "prob_dist_non_match": ...}}}
-- and the JSON written by `save_params_to_json_file` is the reference's
{"current_params", "historical_params", "settings"} document, so saved models load in
either implementation.  The EM updates arrive through `_update_params(λ, rows)` with rows
shaped like the reference's collected π table (maximisation_step.py:82-90).
"""
import copy
import json
import logging
import os

from .settings import complete_settings_dict

logger = logging.getLogger(__name__)



_ATOMS = frozenset((str, int, float, bool, type(None)))


def _copy_tree(x):
    """copy.deepcopy for the params dict (dicts / lists of str, int, float, bool, None), several times
    faster; any other type (a numpy scalar, a dict subclass) goes through copy.deepcopy."""
    t = type(x)
    if t is dict:
        return {k: _copy_tree(v) for k, v in x.items()}
    if t is list:
        return [_copy_tree(v) for v in x]
    if t in _ATOMS:
        return x
    return copy.deepcopy(x)

class Params:
    """Current parameters (`self.params`) plus the value after every EM iteration (`self.param_history`)."""

    def __init__(self, settings: dict, spark):
        self.param_history = []
        self.iteration = 1
        self.settings = complete_settings_dict(settings, spark)
        self.params = {"λ": settings["proportion_of_matches"], "π": {}}
        self.log_likelihood_exists = False
        self.real_params = None
        self._generate_param_dict()

    @property
    def _gamma_cols(self):
        return self.params["π"].keys()

    def describe_gammas(self):
        return {k: v["desc"] for k, v in self.params["π"].items()}

    def _generate_param_dict(self):
        for col in self.settings["comparison_columns"]:
            name = col["col_name"] if "col_name" in col else col["custom_name"]
            entry = {"gamma_index": col["gamma_index"], "desc": f"Comparison of {name}", "column_name": f"{name}"}
            if "custom_name" in col:
                entry["custom_comparison"] = True
                entry["custom_columns_used"] = col["custom_columns_used"]
            else:
                entry["custom_comparison"] = False
            levels = col["num_levels"]
            entry["num_levels"] = levels
            m = [p / sum(col["m_probabilities"]) for p in col["m_probabilities"]]
            u = [p / sum(col["u_probabilities"]) for p in col["u_probabilities"]]
            entry["prob_dist_match"] = {f"level_{i}": {"value": i, "probability": m[i]} for i in range(levels)}
            entry["prob_dist_non_match"] = {f"level_{i}": {"value": i, "probability": u[i]} for i in range(levels)}
            self.params["π"][f"gamma_{name}"] = entry

    def _set_pi_value(self, gamma_str, level_int, match_str, prob_float):
        self.params["π"][gamma_str][f"prob_dist_{match_str}"][f"level_{level_int}"]["probability"] = prob_float

    # ---- level tables for the device ---------------------------------------------------
    def _level_probabilities(self):
        """[(m list, u list)] per gamma column, in gamma order."""
        out = []
        for g in self._gamma_cols:
            d = self.params["π"][g]
            n = d["num_levels"]
            out.append(([d["prob_dist_match"][f"level_{i}"]["probability"] for i in range(n)],
                        [d["prob_dist_non_match"][f"level_{i}"]["probability"] for i in range(n)]))
        return out

    # ---- history / presentation data -----------------------------------------------------
    @staticmethod
    def _convert_params_dict_to_dataframe(params, iteration_num=None):
        rows = []
        for gamma_str, d in params["π"].items():
            for match, key in ((1, "prob_dist_match"), (0, "prob_dist_non_match")):
                for level_str, level in d[key].items():
                    row = {} if iteration_num is None else {"iteration": iteration_num}
                    row.update({"gamma": gamma_str, "match": match, "value_of_gamma": level_str,
                                "probability": level["probability"], "value": level["value"],
                                "column": d["column_name"]})
                    rows.append(row)
        return rows

    def _convert_params_dict_to_normalised_adjustment_data(self):
        rows = []
        for d in self.params["π"].values():
            for i in range(d["num_levels"]):
                lvl = f"level_{i}"
                m = d["prob_dist_match"][lvl]["probability"]
                u = d["prob_dist_non_match"][lvl]["probability"]
                row = {"level": lvl, "col_name": d["column_name"], "m": m, "u": u}
                try:
                    row["adjustment"] = m / (m + u)
                    row["normalised_adjustment"] = row["adjustment"] - 0.5
                except ZeroDivisionError:
                    row["adjustment"] = None
                    row["normalised_adjustment"] = None
                rows.append(row)
        return rows

    def _iteration_history_df_gammas(self):
        rows = []
        n = len(self.param_history)
        for i, p in enumerate(self.param_history):
            rows.extend(self._convert_params_dict_to_dataframe(p, i))
        rows.extend(self._convert_params_dict_to_dataframe(self.params, n))
        return rows

    def _iteration_history_df_lambdas(self):
        rows = [{"λ": p["λ"], "iteration": i} for i, p in enumerate(self.param_history)]
        rows.append({"λ": self.params["λ"], "iteration": len(self.param_history)})
        return rows

    def _iteration_history_df_log_likelihood(self):
        rows = [{"log_likelihood": p["log_likelihood"], "iteration": i} for i, p in enumerate(self.param_history)]
        rows.append({"log_likelihood": self.params["log_likelihood"], "iteration": len(self.param_history)})
        return rows

    # ---- EM update (params.py:225-285) --------------------------------------------------------
    def _reset_param_values_to_none(self):
        self.params["λ"] = None
        for d in self.params["π"].values():
            for key in ("prob_dist_match", "prob_dist_non_match"):
                for level in d[key].values():
                    level["probability"] = None

    def _save_params_to_iteration_history(self):
        self.param_history.append(_copy_tree(self.params))
        if "log_likelihood" in self.params:
            self.log_likelihood_exists = True

    def _populate_params(self, lambda_value, pi_df_collected):
        self.params["λ"] = lambda_value
        for d in self.params["π"].values():  # levels never observed stay at 0
            for key in ("prob_dist_match", "prob_dist_non_match"):
                for level in d[key].values():
                    level["probability"] = 0
        for row in pi_df_collected:
            level = row["gamma_value"]
            if level == -1:
                continue
            self._set_pi_value(row["gamma_col"], level, "match", row["new_probability_match"])
            self._set_pi_value(row["gamma_col"], level, "non_match", row["new_probability_non_match"])

    def _update_params(self, lambda_value, pi_df_collected):
        self._save_params_to_iteration_history()
        self._reset_param_values_to_none()
        self._populate_params(lambda_value, pi_df_collected)
        self.iteration += 1

    # ---- persistence ----------------------------------------------------------------------------
    def _to_dict(self):
        return {"current_params": self.params, "historical_params": self.param_history, "settings": self.settings}

    def save_params_to_json_file(self, path=None, overwrite=False):
        if not path:
            raise ValueError("Must provide a path to write to")
        if os.path.isfile(path) and not overwrite:
            raise ValueError(f"The path {path} already exists. Please provide a different path.")
        with open(path, "w") as f:
            json.dump(self._to_dict(), f, indent=4)

    def is_converged(self):
        """All m/u moved by less than `em_convergence` since the last iteration (params.py:316-336)."""
        new = {k: v for k, v in _flatten_dict(self.params).items() if "_probability" in k.lower()}
        old = {k: v for k, v in _flatten_dict(self.param_history[-1]).items() if "_probability" in k.lower()}
        threshold = self.settings["em_convergence"]
        ok = [abs(new[k] - old[k]) < threshold for k in new]
        biggest, biggest_key = 0, ""
        for k in new:
            change = abs(new[k] - old[k])
            if change > biggest:
                biggest, biggest_key = change, k
        logger.info(f"The maximum change in parameters was {biggest} for key {biggest_key}")
        return all(ok)

    # ---- presentation (out of scope for the GPU path; data only) ------------------------------
    def _print_m_u_probs(self):
        for field, d in self.params["π"].items():
            print(field)
            print(f'"m_probabilities": {[v["probability"] for v in d["prob_dist_match"].values()]},')
            print(f'"u_probabilities": {[v["probability"] for v in d["prob_dist_non_match"].values()]}')

    def _chart(self, title, data, x, y, color=None):
        spec = {"$schema": "https://vega.github.io/schema/vega-lite/v3.json", "title": title,
                "data": {"values": data}, "mark": "bar",
                "encoding": {"x": {"field": x, "type": "nominal"}, "y": {"field": y, "type": "quantitative"}}}
        if color:
            spec["encoding"]["color"] = {"field": color, "type": "nominal"}
        return spec

    def probability_distribution_chart(self):
        return self._chart("Probability distribution of gamma values",
                           self._convert_params_dict_to_dataframe(self.params), "value_of_gamma", "probability",
                           "match")

    def adjustment_factor_chart(self):
        return self._chart("Adjustment factors", self._convert_params_dict_to_normalised_adjustment_data(), "level",
                           "normalised_adjustment", "col_name")

    def lambda_iteration_chart(self):
        return self._chart("λ by iteration", self._iteration_history_df_lambdas(), "iteration", "λ")

    def pi_iteration_chart(self):
        return self._chart("π by iteration", self._iteration_history_df_gammas(), "iteration", "probability",
                           "gamma")

    def ll_iteration_chart(self):
        if not self.log_likelihood_exists:
            raise Exception("Log likelihood not calculated.  To calculate pass 'compute_ll=True' to iterate(). "
                            "Note this causes algorithm to run more slowly because additional calculations are "
                            "required.")
        return self._chart("Log likelihood by iteration", self._iteration_history_df_log_likelihood(), "iteration",
                           "log_likelihood")

    def __repr__(self):  # pragma: no cover
        p = self.params
        lines = [f"λ (proportion of matches) = {p['λ']}"]
        for gamma_str, d in p["π"].items():
            lines += ["------------------------------------", f"{gamma_str}: {d['desc']}", ""]
            for title, key in (("matches", "prob_dist_match"), ("non-matches", "prob_dist_non_match")):
                lines.append(f"Probability distribution of gamma values amongst {title}:")
                for level in d[key].values():
                    prob = level["probability"]
                    lines.append(f"    value {level['value']}: {'None' if not prob else f'{prob:4f}'}")
                lines.append("")
        return "\n".join(lines)


def load_params_from_json(path):
    with open(path, "r") as f:
        return load_params_from_dict(json.load(f))


def load_params_from_dict(param_dict):
    if set(param_dict.keys()) != {"current_params", "settings", "historical_params"}:
        raise ValueError("Your saved params seem to be corrupted")
    p = Params(settings=param_dict["settings"], spark=None)
    p.params = param_dict["current_params"]
    p.param_history = param_dict["historical_params"]
    return p


def _flatten_dict(dictionary, accumulator=None, parent_key=None, separator="_"):
    if accumulator is None:
        accumulator = {}
    for k, v in dictionary.items():
        key = f"{parent_key}{separator}{k}" if parent_key else k
        if isinstance(v, dict):
            _flatten_dict(v, accumulator, key)
        else:
            accumulator[key] = v
    return accumulator
