"""HTML wrappers for the chart table (presentation; reference
simulation_utils.py:115-316). One row builder, two page styles: a
full-viewport table scrolled by dragging, and a notebook-friendly table."""

from __future__ import annotations

import pandas as pd

_CELL_CSS = """
    table { border-collapse: collapse; margin: 0; width: auto; }
    td, th { padding: 10px; vertical-align: top; text-align: center; }
    .case-group-even td { background-color: #FFFFFF !important; }
"""

_DRAG_CSS = """<style>
    body { margin: 0; padding: 0; overflow: hidden; }
    .scrollable-table-container { background-color: #FFFFFF; width: 100%; height: 100vh;
        overflow: auto; border: 1px solid #ccc; position: relative; user-select: none; cursor: grab; }
    .scrollable-table-container:active { cursor: grabbing; }
    .scrollable-table-container img { user-select: none; -webkit-user-drag: none; pointer-events: none; }
    .case-group-odd td { background-color: #F0F0F0 !important; }""" + _CELL_CSS + "</style>"

_DRAG_JS = """<script>
document.addEventListener('DOMContentLoaded', () => {
  const box = document.querySelector('.scrollable-table-container');
  let drag = null;
  box.addEventListener('dragstart', ev => ev.preventDefault());
  box.addEventListener('mousedown', ev => {
    ev.preventDefault();
    drag = {x: ev.clientX, y: ev.clientY, left: box.scrollLeft, top: box.scrollTop};
  });
  document.addEventListener('mouseup', () => { drag = null; });
  document.addEventListener('mousemove', ev => {
    if (!drag) return;
    ev.preventDefault();
    box.scrollLeft = drag.left - (ev.clientX - drag.x);
    box.scrollTop = drag.top - (ev.clientY - drag.y);
  });
});
</script>"""

_NOTEBOOK_CSS = """<style>
    .scrollable-table-container { background-color: #FFFFFF; width: 100%; overflow-x: auto;
        overflow-y: hidden; white-space: nowrap; border: 1px solid #ccc; }
    .case-group-odd td { background-color: #F8F8F8 !important; }""" + _CELL_CSS + "</style>"


def _rows_html(table_data: dict[str, list[str]], summary_table: pd.DataFrame,
               case_row_ranges: list[tuple[int, int, int]]) -> str:
    def case_of(row: int) -> int:
        return next((c for start, end, c in case_row_ranges if start <= row <= end), 0)

    n_rows = len(next(iter(table_data.values())))
    cols = list(summary_table.columns)
    body = []
    for i in range(n_rows):
        cls = "case-group-even" if case_of(i) % 2 == 0 else "case-group-odd"
        cells = "".join(f"<td>{summary_table[c][i]}</td>" for c in cols)
        body.append(f"<tr class='{cls}'>{cells}</tr>")
    head = "".join(f"<th>{c}</th>" for c in cols)
    return (f'<div class="scrollable-table-container"><table><thead><tr>{head}</tr></thead>'
            f"<tbody>{''.join(body)}</tbody></table></div>")


def _generate_draggable_html_table(table_data, summary_table, case_row_ranges) -> str:
    return _DRAG_CSS + _DRAG_JS + _rows_html(table_data, summary_table, case_row_ranges)


def _generate_ipynb_table(table_data, summary_table, case_row_ranges) -> str:
    return _NOTEBOOK_CSS + _rows_html(table_data, summary_table, case_row_ranges)
