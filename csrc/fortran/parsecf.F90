! Fortran 2008 bindings of the parsec-amd C API (include/parsec.h).
! Same module surface as the reference's parsec/fortran/parsecf.F90
! (parsec_init / fini / compose / context add-start-test-wait / taskpool
! callbacks / version), plus DTD task insertion through the varargs-free
! parsec_dtd_insert_task_array so Fortran programs can build task graphs.
module parsec_f08
  use, intrinsic :: iso_c_binding
  implicit none

  type, bind(C) :: parsec_taskpool_t
    type(c_ptr) :: ptr = c_null_ptr
  end type parsec_taskpool_t

  type, bind(C) :: parsec_context_t
    type(c_ptr) :: ptr = c_null_ptr
  end type parsec_context_t

  integer(c_int), parameter :: PARSEC_SUCCESS = 0
  integer(c_int), parameter :: PARSEC_HOOK_RETURN_DONE = 0
  integer(c_int), parameter :: PARSEC_DEV_CPU = 1
  integer(c_int), parameter :: PARSEC_INPUT = int(z'100000', c_int)
  integer(c_int), parameter :: PARSEC_OUTPUT = int(z'200000', c_int)
  integer(c_int), parameter :: PARSEC_INOUT = int(z'300000', c_int)
  integer(c_int), parameter :: PARSEC_VALUE = int(z'600000', c_int)

  abstract interface
    function parsec_event_cb(tp, cbdata) bind(C) result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: tp
      type(c_ptr), value :: cbdata
      integer(c_int) :: rc
    end function parsec_event_cb
    function parsec_dtd_body(es, task) bind(C) result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: es
      type(c_ptr), value :: task
      integer(c_int) :: rc
    end function parsec_dtd_body
  end interface

  interface
    function parsec_version_f08(major, minor, patch) bind(C, name="parsec_version") result(rc)
      import :: c_int
      integer(c_int), intent(out) :: major, minor, patch
      integer(c_int) :: rc
    end function parsec_version_f08
    function parsec_version_ex_c(len, str) bind(C, name="parsec_version_ex") result(rc)
      import :: c_int, c_size_t, c_char
      integer(c_size_t), value :: len
      character(kind=c_char), dimension(*) :: str
      integer(c_int) :: rc
    end function parsec_version_ex_c
    subroutine parsec_init_f08(nbcores, ctx, ierr) bind(C, name="parsec_init_f08")
      import :: c_int, parsec_context_t
      integer(c_int), value :: nbcores
      type(parsec_context_t), intent(out) :: ctx
      integer(c_int), intent(out) :: ierr
    end subroutine parsec_init_f08
    subroutine parsec_fini_f08(ctx, ierr) bind(C, name="parsec_fini_f08")
      import :: c_int, parsec_context_t
      type(parsec_context_t), intent(inout) :: ctx
      integer(c_int), intent(out) :: ierr
    end subroutine parsec_fini_f08
    function parsec_compose_f08(start, next) bind(C, name="parsec_compose") result(tp)
      import :: parsec_taskpool_t
      type(parsec_taskpool_t), value :: start, next
      type(parsec_taskpool_t) :: tp
    end function parsec_compose_f08
    subroutine parsec_taskpool_free_f08(tp) bind(C, name="parsec_taskpool_free")
      import :: parsec_taskpool_t
      type(parsec_taskpool_t), value :: tp
    end subroutine parsec_taskpool_free_f08
    function parsec_context_add_taskpool_f08(ctx, tp) bind(C, name="parsec_context_add_taskpool") result(rc)
      import :: c_int, parsec_context_t, parsec_taskpool_t
      type(parsec_context_t), value :: ctx
      type(parsec_taskpool_t), value :: tp
      integer(c_int) :: rc
    end function parsec_context_add_taskpool_f08
    function parsec_context_start_f08(ctx) bind(C, name="parsec_context_start") result(rc)
      import :: c_int, parsec_context_t
      type(parsec_context_t), value :: ctx
      integer(c_int) :: rc
    end function parsec_context_start_f08
    function parsec_context_test_f08(ctx) bind(C, name="parsec_context_test") result(rc)
      import :: c_int, parsec_context_t
      type(parsec_context_t), value :: ctx
      integer(c_int) :: rc
    end function parsec_context_test_f08
    function parsec_context_wait_f08(ctx) bind(C, name="parsec_context_wait") result(rc)
      import :: c_int, parsec_context_t
      type(parsec_context_t), value :: ctx
      integer(c_int) :: rc
    end function parsec_context_wait_f08
    function parsec_taskpool_set_complete_callback_c(tp, cb, cbdata) bind(C, name="parsec_taskpool_set_complete_callback") result(rc)
      import :: c_int, c_funptr, c_ptr, parsec_taskpool_t
      type(parsec_taskpool_t), value :: tp
      type(c_funptr), value :: cb
      type(c_ptr), value :: cbdata
      integer(c_int) :: rc
    end function parsec_taskpool_set_complete_callback_c
    function parsec_taskpool_set_enqueue_callback_c(tp, cb, cbdata) bind(C, name="parsec_taskpool_set_enqueue_callback") result(rc)
      import :: c_int, c_funptr, c_ptr, parsec_taskpool_t
      type(parsec_taskpool_t), value :: tp
      type(c_funptr), value :: cb
      type(c_ptr), value :: cbdata
      integer(c_int) :: rc
    end function parsec_taskpool_set_enqueue_callback_c
    subroutine parsec_taskpool_get_complete_callback_f08(tp, cb, cbdata, ierr) bind(C, name="parsec_taskpool_get_complete_callback_f08")
      import :: c_int, c_funptr, c_ptr, parsec_taskpool_t
      type(parsec_taskpool_t), value :: tp
      type(c_funptr), intent(out) :: cb
      type(c_ptr), intent(out) :: cbdata
      integer(c_int), intent(out) :: ierr
    end subroutine parsec_taskpool_get_complete_callback_f08
    subroutine parsec_taskpool_get_enqueue_callback_f08(tp, cb, cbdata, ierr) bind(C, name="parsec_taskpool_get_enqueue_callback_f08")
      import :: c_int, c_funptr, c_ptr, parsec_taskpool_t
      type(parsec_taskpool_t), value :: tp
      type(c_funptr), intent(out) :: cb
      type(c_ptr), intent(out) :: cbdata
      integer(c_int), intent(out) :: ierr
    end subroutine parsec_taskpool_get_enqueue_callback_f08
    function parsec_taskpool_set_priority_f08(tp, prio) bind(C, name="parsec_taskpool_set_priority") result(old)
      import :: c_int32_t, parsec_taskpool_t
      type(parsec_taskpool_t), value :: tp
      integer(c_int32_t), value :: prio
      integer(c_int32_t) :: old
    end function parsec_taskpool_set_priority_f08
    ! DTD
    function parsec_dtd_taskpool_new_f08() bind(C, name="parsec_dtd_taskpool_new") result(tp)
      import :: parsec_taskpool_t
      type(parsec_taskpool_t) :: tp
    end function parsec_dtd_taskpool_new_f08
    subroutine parsec_dtd_taskpool_wait_f08(tp) bind(C, name="parsec_dtd_taskpool_wait")
      import :: parsec_taskpool_t
      type(parsec_taskpool_t), value :: tp
    end subroutine parsec_dtd_taskpool_wait_f08
    subroutine parsec_dtd_insert_task_array_c(tp, body, prio, devtype, name, nargs, sizes, ptrs, flags) &
        bind(C, name="parsec_dtd_insert_task_array")
      import :: c_int, c_funptr, c_ptr, c_char, parsec_taskpool_t
      type(parsec_taskpool_t), value :: tp
      type(c_funptr), value :: body
      integer(c_int), value :: prio, devtype
      character(kind=c_char), dimension(*) :: name
      integer(c_int), value :: nargs
      integer(c_int), dimension(*) :: sizes
      type(c_ptr), dimension(*) :: ptrs
      integer(c_int), dimension(*) :: flags
    end subroutine parsec_dtd_insert_task_array_c
    function parsec_dtd_task_arg_f08(task, i) bind(C, name="parsec_dtd_task_arg") result(p)
      import :: c_ptr, c_int
      type(c_ptr), value :: task
      integer(c_int), value :: i
      type(c_ptr) :: p
    end function parsec_dtd_task_arg_f08
  end interface

contains

  subroutine parsec_version_ex_f08(str, ierr)
    character(len=*), intent(out) :: str
    integer(c_int), intent(out) :: ierr
    character(kind=c_char), dimension(len(str) + 1) :: buf
    integer :: i
    buf = c_null_char
    ierr = parsec_version_ex_c(int(len(str) + 1, c_size_t), buf)
    str = ' '
    do i = 1, len(str)
      if (buf(i) == c_null_char) exit
      str(i:i) = buf(i)
    end do
  end subroutine parsec_version_ex_f08

  subroutine parsec_taskpool_set_complete_callback_f08(tp, cb, cbdata, ierr)
    type(parsec_taskpool_t), intent(in) :: tp
    procedure(parsec_event_cb) :: cb
    type(c_ptr), intent(in) :: cbdata
    integer(c_int), intent(out) :: ierr
    ierr = parsec_taskpool_set_complete_callback_c(tp, c_funloc(cb), cbdata)
  end subroutine parsec_taskpool_set_complete_callback_f08

  subroutine parsec_taskpool_set_enqueue_callback_f08(tp, cb, cbdata, ierr)
    type(parsec_taskpool_t), intent(in) :: tp
    procedure(parsec_event_cb) :: cb
    type(c_ptr), intent(in) :: cbdata
    integer(c_int), intent(out) :: ierr
    ierr = parsec_taskpool_set_enqueue_callback_c(tp, c_funloc(cb), cbdata)
  end subroutine parsec_taskpool_set_enqueue_callback_f08

  ! Insert a DTD task: args are described by parallel arrays (size in bytes
  ! for PARSEC_VALUE, flags = access mode | affinity bits, pointer = value
  ! address or tile handle).
  subroutine parsec_dtd_insert_task_f08(tp, body, prio, devtype, name, sizes, ptrs, flags)
    type(parsec_taskpool_t), intent(in) :: tp
    procedure(parsec_dtd_body) :: body
    integer(c_int), intent(in) :: prio, devtype
    character(len=*), intent(in) :: name
    integer(c_int), dimension(:), intent(in) :: sizes, flags
    type(c_ptr), dimension(:), intent(in) :: ptrs
    integer(c_int), dimension(size(sizes)) :: s, f
    type(c_ptr), dimension(size(sizes)) :: p
    s = sizes
    f = flags
    p = ptrs
    call parsec_dtd_insert_task_array_c(tp, c_funloc(body), prio, devtype, trim(name) // c_null_char, &
                                        int(size(sizes), c_int), s, p, f)
  end subroutine parsec_dtd_insert_task_f08

end module parsec_f08
