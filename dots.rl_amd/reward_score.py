"""Rule-based reward scoring (mirror of verl/utils/reward_score/__init__.py:19-123 and gsm8k.py:19-72).

Only the data sources on this repository's path are implemented: ``openai/gsm8k`` (config #1). Other
sources raise NotImplementedError exactly as the reference does for a source it does not know.
"""

from __future__ import annotations

import re

_SOLUTION_CLIP_CHARS = 300
_STRICT = re.compile("#### (\\-?[0-9\\.\\,]+)")
_FLEXIBLE = re.compile("(\\-?[0-9\\.\\,]+)")


def gsm8k_extract_solution(solution_str: str, method: str = "strict"):
    """gsm8k.py:20-50: the last '#### <number>' (strict) or the last number that is not '' / '.' (flexible),
    searched in the final 300 characters; commas and '$' removed in strict mode."""
    assert method in ["strict", "flexible"]
    if len(solution_str) > _SOLUTION_CLIP_CHARS:
        solution_str = solution_str[-_SOLUTION_CLIP_CHARS:]
    if method == "strict":
        found = _STRICT.findall(solution_str)
        return found[-1].replace(",", "").replace("$", "") if found else None
    final = None
    for final in reversed(_FLEXIBLE.findall(solution_str)):
        if final not in ("", "."):
            break
    return final


def gsm8k_compute_score(solution_str, ground_truth, method="strict", format_score=0.0, score=1.0):
    """gsm8k.py:53-72: `score` for the right answer, `format_score` for a wrong one, 0 with no answer."""
    answer = gsm8k_extract_solution(solution_str=solution_str, method=method)
    if answer is None:
        return 0
    return score if answer == ground_truth else format_score


def default_compute_score(data_source, solution_str, ground_truth, extra_info=None, sandbox_fusion_url=None,
                          concurrent_semaphore=None, memory_limit_mb=None):
    """reward_score/__init__.py:19-114 for the sources on this path; float result (a dict passes through)."""
    if data_source == "openai/gsm8k":
        res = gsm8k_compute_score(solution_str, ground_truth)
    else:
        raise NotImplementedError(f"Reward function is not implemented for {data_source=}")
    if isinstance(res, dict):
        return res
    if isinstance(res, (int, float, bool)):
        return float(res)
    return float(res[0])
